#!/usr/bin/env python3
"""Static instruction mix of the loops of one classify2_kernel instance.
Usage: asm_loops.py FILE.s [TEMPLATE_BITS]   (bits: HIST COMPACT REMAP BIN FLAG,
default 01011 = the binned flagged kernel).  FILE.s from
hipcc --cuda-device-only -S."""
import re
import sys

path = sys.argv[1]
want = tuple(sys.argv[2]) if len(sys.argv) > 2 else tuple("01011")
s = open(path).read()
parts = re.split(r"^(_Z\S+):\s*(?:;.*)?$", s, flags=re.M)
for i in range(1, len(parts), 2):
    name, body = parts[i], parts[i + 1]
    if "classify2" not in name:
        continue
    if re.search(r"ILb(\d)ELb(\d)ELb(\d)ELb(\d)ELb(\d)E", name).groups() != want:
        continue
    body = body.split(".Lfunc_end")[0]
    meta = {k: (re.search(r";\s*%s:\s*(\d+)" % k, parts[i + 1]) or [0, "?"])[1]
            for k in ("NumVgprs", "NumSgprs", "ScratchSize")}
    print(name[:60], meta)
    lines = body.split("\n")
    labels = {}
    for n, l in enumerate(lines):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = n
    seen = set()
    for n, l in enumerate(lines):
        m = re.search(r"s_c?branch\S*\s+(\.LBB\S+)", l)
        if not (m and labels.get(m.group(1), 1 << 30) < n):
            continue
        a = labels[m.group(1)]
        seg = [x.strip().split()[0] for x in lines[a:n]
               if x.startswith("\t") and not x.strip().startswith((".", ";"))]
        if len(seg) < 150 or a in seen:
            continue
        seen.add(a)
        cnt = lambda p: sum(1 for x in seg if x.startswith(p))
        print(f"loop lines {a}-{n}: ins {len(seg)} valu {cnt('v_')} salu {cnt('s_')} "
              f"lane-rw {cnt('v_writelane') + cnt('v_readlane')} ds {cnt('ds_')} cmp {cnt('v_cmp')}")

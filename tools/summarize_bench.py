#!/usr/bin/env python3
"""One bench.py line -> the numbers a run is judged on (tools/gpu_run.sh)."""
import json
import sys

for path in sys.argv[1:]:
    lines = [ln for ln in open(path) if ln.startswith("{")]
    if not lines:
        print(path, "no JSON line")
        continue
    d = json.loads(lines[-1])
    r = d.get("roofline") or {}
    k = d.get("kernels_ms_per_step") or {}
    sd = d.get("step_driver") or {}
    print(path, "ms/step", d["ms_per_step"], "n_gpus", d["n_gpus"], "parity", d.get("parity"),
          "frac", r.get("frac"), r.get("kernel"), r.get("avg_launch_ms"))
    print("  single_batch_ms", d.get("single_batch_ms"), "parity_detail",
          {x: (d.get("parity_detail") or {}).get(x) for x in ("against", "mismatch", "edges")},
          "timed_step", ((d.get("parity_detail") or {}).get("timed_step") or {}).get("deferred_on_every_rank"))
    print("  transport", d.get("transport"))
    print("  host_us", d.get("host_us_per_step"), "calls", d.get("api_calls_per_step"), "wait_us",
          sd.get("host_wait_us_per_step"), "drain_us", sd.get("drain_us"), "mode", sd.get("mode"))
    print("  kernels", {x: k[x] for x in sorted(k, key=lambda x: -k[x]) if k[x] > 0.005})
    for key in ("profile_write_ceiling", "eq_path", "dropin", "cpu_baseline", "vs_reference_measured", "weak"):
        v = d.get(key)
        if isinstance(v, dict):
            v = {x: v[x] for x in v if x in ("ms", "seconds", "value", "profile_vs_ceiling", "profile_ms",
                                             "memset_ms", "speedup_vs_reference", "ms_per_step", "cores")}
        if v is not None:
            print("  ", key, v)

#!/usr/bin/env python3
"""Golden vectors for the host parsers (csrc/ingest.cpp), captured by running the
REFERENCE in this container (never on the GPU box).  Writes tests/golden/ingest.json.

  fasta  karma/karma.py:40-61 read_fasta_file.  karma.py itself does not import
         (numba.errors, circular import: SURVEY.md §8(c)), so the function's
         own definition is taken from karma.py's syntax tree and executed with
         OrderedDict and a silent logger in its namespace.
  eq     ReadGraph.from_equivalence_classes (read_graph.py:61-148) on
         parse-focused eq_classes.txt texts (graph or exception name).
  sam    SAM lines grouped by RNAME in order of first appearance (the bulk
         helper's contract, contig.py has no grouping of its own), each group
         through Contig.load_from_iterator (contig.py:29-35), then
         ReadGraph.from_contigs (read_graph.py:19-50).

File texts are stored as hex so that invalid UTF-8 and lone "\\r" survive JSON.
Usage:  python tests/golden/make_golden_ingest.py
"""
import ast
import json
import logging
import os
import sys
from collections import OrderedDict

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from make_golden import REF, eq_case, graph_dump, import_reference  # noqa: E402


def reference_read_fasta_file():
    src = open(os.path.join(REF, "karma", "karma.py")).read()
    tree = ast.parse(src)
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "read_fasta_file")
    ns = {"OrderedDict": OrderedDict, "logger": logging.getLogger("karma_ref_silent")}
    ns["logger"].setLevel(logging.CRITICAL)
    exec(compile(ast.Module(body=[fn], type_ignores=[]), "karma.py", "exec"), ns)
    return ns["read_fasta_file"]


FASTA = OrderedDict()
FASTA["basic"] = b">c1 desc\nACGT\nAC\n>c2\nGG\n"
FASTA["crlf"] = b">a x\r\nAC\r\nGT\r\n>b\r\nTT\r\n"
FASTA["lone_cr"] = b">a\rAC\rGT\r>b\rN\r"
FASTA["no_header_first_line"] = b"ACGT\nTT\n>b\nGG"
FASTA["empty"] = b""
FASTA["only_newline"] = b"\n"
FASTA["dup_keys"] = b">a\nAA\n>b\nCC\n>a\nGG\n>b x\n"
FASTA["gt_midline"] = b">a\nAC>GT\n >x\n>b\nT"
FASTA["tabs_spaces"] = b">a\tb c\nA C\tG\n>\n>  \nAC"
FASTA["utf8"] = ">ключ é\nACGTé\n>b\nGG\n".encode("utf-8")
FASTA["blank_lines"] = b">a\n\nAC\n\n>b\n\n"
FASTA["last_header_no_body"] = b">a\nAC\n>b"
FASTA["cr_crlf_mix"] = b">a\r\r\nAC\n\rGT\r\n\n>b\r>c"
FASTA["nul_and_lower"] = b">n\x00m\nacg\x00t\n"
FASTA["invalid_utf8"] = b">a\nAC\xffGT\n"
FASTA["truncated_utf8"] = b">a\nAC\xc3"

EQ = OrderedDict()
EQ["underscore_count"] = ("2\n1\na\nb\n2\t0\t1\t1_0\n", [">a", ">b"])
EQ["spaced_count"] = ("2\n1\na\nb\n2\t0\t1\t 7 \n2\t1\t0\t\t3\n", [">a", ">b"])
EQ["tab_padded_count"] = ("2\n1\na\nb\n2\t0\t1\t\t3\n", [">a", ">b"])
EQ["leading_zero_id"] = ("2\n1\na\nb\n2\t00\t1\t5\n", [">a", ">b"])
EQ["plus_id"] = ("2\n1\na\nb\n2\t+0\t1\t5\n", [">a", ">b"])
EQ["empty_line"] = ("2\n1\na\nb\n2\t0\t1\t5\n\n", [">a", ">b"])
EQ["one_field"] = ("2\n1\na\nb\n5\n", [">a", ">b"])
EQ["bad_count"] = ("2\n1\na\nb\n2\t0\t1\t5x\n", [">a", ">b"])
EQ["double_underscore"] = ("2\n1\na\nb\n2\t0\t1\t1__0\n", [">a", ">b"])
EQ["names_past_eof"] = ("3\n0\na\n", [">a", ">b"])
EQ["header_spaces"] = (" 3 \n9\nx y\nz\nw\n2\t0\t2\t4\n2\t1\t2\t6\n", [">x y", ">z", ">w"])
EQ["crlf_everywhere"] = ("2\r\n1\r\na\r\nb\r\n2\t0\t1\t5\r\n", [">a", ">b"])
EQ["lone_cr"] = ("2\r1\ra\rb\r2\t0\t1\t5\r1\t1\t2\r", [">a", ">b"])
EQ["size_token_01"] = ("2\n1\na\nb\n01\t0\t1\t5\n", [">a", ">b"])
EQ["utf8_names"] = ("2\n1\nα\nβ\n2\t0\t1\t5\n", [">α", ">β"])
EQ["negative_n"] = ("-1\n0\n", [">a"])
EQ["bad_header"] = ("x\n0\n", [">a"])
EQ["zero_contigs"] = ("0\n0\n", [])

SAM = OrderedDict()
SAM["basic"] = b"r1\t0\tc1\t5\t60\t*\nr1\t16\tc2\t9\nr2\t0\tc1\t1\nr3\t0\tc2\t1\nr2\t0\tc3\t7\tx\n"
SAM["headers"] = b"@HD\tVN:1.6\n@SQ\tSN:c1\tLN:9\nq\t0\tc1\t1\nq\t0\tc2\t1\np\t0\tc2\t1\n"
SAM["crlf_dupes"] = b"a\t0\tx\t1\r\na\t16\tx\t3\r\nb\t0\ty\t1\r\na\t0\ty\t4\r\n"
SAM["one_contig"] = b"r\t0\tonly\t1\n"
SAM["too_few_fields"] = b"r1\t0\tc1\t1\nr2\t0\tc1\n"


def main():
    KC, RG, Contig, scratch = import_reference()
    rff = reference_read_fasta_file()
    out = {"generator": "tests/golden/make_golden_ingest.py", "reference": "lmfaber/karma (v0)"}

    fa = {}
    for name, data in FASTA.items():
        path = os.path.join(scratch, f"{name}.fa")
        with open(path, "wb") as f:
            f.write(data)
        try:
            d = rff(path)
            res = {"items": [[k, v] for k, v in d.items()]}
        except Exception as e:  # e.g. UnicodeDecodeError
            res = {"raises": type(e).__name__}
        fa[name] = {"hex": data.hex(), "out": res}
    out["fasta"] = fa

    out["eq"] = {k: {"hex": t.encode("utf-8").hex(), "fasta": f, "out": eq_case(RG, t, f, scratch, k)}
                 for k, (t, f) in EQ.items()}

    sm = {}
    for name, data in SAM.items():
        lines = data.decode("utf-8").splitlines()
        lines = [ln for ln in lines if not ln.startswith("@")]  # hisat2.py:49-53
        groups = OrderedDict()
        try:
            for ln in lines:
                rname = ln.split("\t")[2]
                groups.setdefault(rname, []).append(ln)
        except IndexError:
            groups = None
        res = {}
        try:
            if groups is None:
                raise ValueError("fewer than 3 fields")
            contigs = []
            for rname, ls in groups.items():
                c = Contig(rname)
                c.load_from_iterator(ls)
                contigs.append(c)
            res["readsets"] = [[c.name, sorted(c.readset)] for c in contigs]
            res["graph"] = graph_dump(RG.from_contigs(contigs))
        except Exception as e:
            res = {"raises": type(e).__name__}
        sm[name] = {"hex": data.hex(), "out": res}
    out["sam"] = sm

    path = os.path.join(HERE, "ingest.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, ensure_ascii=True)
    print("wrote", path)


if __name__ == "__main__":
    main()

"""Known-answer-test runner shared by the CPU (oracle) and GPU (product) parity tests.

A fixture (tests/golden/kats.json) holds the QL app, the InputHandler timeline of a reference
TestNG case and the values that case asserts.  `run_app` replays the timeline against any
engine exposing the reference's test idiom (add_query_callback / add_stream_callback / start /
send / sleep / outputs).
"""
from __future__ import annotations

import json
import math
import os
import struct
from typing import Any, Dict, List

HERE = os.path.dirname(os.path.abspath(__file__))


def load_kats(name: str = "kats.json") -> List[Dict[str, Any]]:
    return json.load(open(os.path.join(HERE, "golden", name)))


def rtc_sample(kats: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    """The KATs the default GPU suite runs through the queries' compiled kernels (test_gpu_nfa_rtc.py), and that
    tools/rtc_precompile.py --suite compiles beforehand: every fortieth, plus the first two of every test class (each
    NFA class -- Count, Logical, Every, Within, Complex, Sequence, the absent ones, the partitions -- is represented;
    KATs on other paths skip)."""
    out, seen, per = [], set(), {}
    for i, k in enumerate(kats):
        cls = k["name"].split(".")[0]
        per[cls] = per.get(cls, 0) + 1
        if (i % 40 == 0 or per[cls] <= 2) and k["name"] not in seen:
            seen.add(k["name"])
            out.append(k)
    return out


def decode_input(v):
    if isinstance(v, dict):
        return v.get("f32", v.get("f64"))
    return v


def run_app(engine, kat) -> List[Dict[str, Any]]:
    for cb in kat["callbacks"]:
        if "query" in cb:
            engine.add_query_callback(cb["query"])
        else:
            engine.add_stream_callback(cb["stream"])
    engine.start()
    for op in kat["ops"]:
        if op[0] == "sleep":
            engine.sleep(op[1])
        elif op[0] == "send":
            engine.send(op[1], [decode_input(v) for v in op[3]], op[2])
        elif op[0] == "send_batch":
            engine.send_many(op[1], [(t, [decode_input(v) for v in d]) for t, d in op[2]], batch=True)
    return engine.outputs()


def value_eq(expected, actual) -> bool:
    if isinstance(expected, dict):
        if "f32" in expected:
            if not isinstance(actual, float):
                return False
            e = struct.unpack("<f", struct.pack("<f", expected["f32"]))[0]
            return e == actual or (math.isnan(e) and math.isnan(actual))
        e = expected["f64"]
        if not isinstance(actual, float):
            return False
        return e == actual or abs(e - actual) <= 1e-9 * max(1.0, abs(e))
    if isinstance(expected, bool) or isinstance(actual, bool):
        return expected is actual or expected == actual
    if isinstance(expected, int) and isinstance(actual, float):
        return False
    return expected == actual


def check(kat, outputs) -> List[str]:
    """Compare engine outputs with the fixture's expectations; return a list of problems."""
    problems = []
    exp = kat["expect"]
    cb_names = [list(c.values())[0] for c in kat["callbacks"]]
    mine = [o for o in outputs if o["name"] in cb_names]
    ins = [r for o in mine for r in o["in"]]
    rms = [r for o in mine for r in o["rm"]]
    if "in_count" in exp and len(ins) != exp["in_count"]:
        problems.append(f"in_count {len(ins)} != {exp['in_count']}")
    if "rm_count" in exp and len(rms) != exp["rm_count"]:
        problems.append(f"rm_count {len(rms)} != {exp['rm_count']}")
    if "arrived" in exp and exp["arrived"] and not mine:
        problems.append("expected events to arrive")
    if "arrived" in exp and exp["arrived"] is False and (ins or rms):
        problems.append("expected no events")
    rows = exp.get("rows", [])
    pool = exp.get("row_source", "in")
    src = ins if pool == "in" else (rms if pool == "rm" else [r for o in mine for r in o["in"] + o["rm"]])
    if exp.get("rows_match") == "set":
        left = list(src)
        for r in rows:
            hit = next((i for i, a in enumerate(left) if len(a) == len(r) and all(value_eq(e, x) for e, x in zip(r, a))), None)
            if hit is None:
                problems.append(f"row {r} not found")
            else:
                left.pop(hit)
    else:
        for i, r in enumerate(rows):
            if i >= len(src):
                problems.append(f"missing row {i}: {r}")
                break
            a = src[i]
            if len(a) != len(r) or not all(value_eq(e, x) for e, x in zip(r, a)):
                problems.append(f"row {i}: expected {r} got {a}")
    for key in ("col_seq", "col_in"):
        if key in exp:
            col, vals = exp[key]["col"], exp[key]["values"]
            got = [r[col] for o in mine for r in o["in"] + o["rm"]]
            if key == "col_seq" and got != vals:
                problems.append(f"column {col} sequence {got} != {vals}")
            if key == "col_in" and (not got or any(v not in vals for v in got)):
                problems.append(f"column {col} values {got} not all in {vals}")
    if "calls" in exp:
        got = [len(o["in"]) + (len(o["rm"]) if o["kind"] == "stream" else 0) for o in mine]
        if got != exp["calls"]:
            problems.append(f"callback grouping {got} != {exp['calls']}")
    return problems

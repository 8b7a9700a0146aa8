"""The C ABI driven from committed descriptors alone (no Python QL front end), on a host without a GPU:
the way the Java shim calls it.  sg_app_create validates and lowers every query
without touching the device; an unsupported query reports SG_E_UNSUPPORTED per query instead of
failing the app (include/siddhi_gfx.h)."""
import ctypes as C
import glob
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "siddhi_amd", "_build", "libsiddhi_gfx.so")
DESC = os.path.join(ROOT, "tests", "golden", "descriptors")
SCHEMA = os.path.join(ROOT, "include", "siddhi_gfx_descriptor.schema.json")
PATH = {1: "followed_by", 2: "nfa", 3: "window_agg", 4: "keyed_followed_by", 5: "window", -2: "unsupported"}
EXPECT = {
    "config1": {"query1": "followed_by"},
    "config2": {"query1": "window_agg"},
    "config3": {"query1": "nfa"},
    "config4": {"query1": "keyed_followed_by"},
    "config5": {"window": "window_agg", "query1": "nfa"},
    "partial": {"ok": "followed_by", "agg": "unsupported"},
    # @purge (not playback): the window query cleans idle keys on the general path; the keyed shape's
    # purge could clean live partials, so it leaves the scan path for the NFA lanes
    "purge": {"win": "window", "keyed": "nfa"},
}


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(LIB):   # built by __graft_entry__.build() / tests/test_abi_cpu.py
        import subprocess
        import sys
        subprocess.check_call([sys.executable, os.path.join(ROOT, "siddhi_amd", "build.py")])
    L = C.CDLL(LIB)
    L.sg_app_create.argtypes = [C.c_char_p, C.c_void_p, C.POINTER(C.c_void_p)]
    L.sg_app_destroy.argtypes = [C.c_void_p]
    L.sg_last_error.restype = C.c_char_p
    L.sg_query_index.argtypes = [C.c_void_p, C.c_char_p]
    L.sg_query_path.argtypes = [C.c_void_p, C.c_int]
    L.sg_query_unsupported_reason.argtypes = [C.c_void_p, C.c_int]
    L.sg_query_unsupported_reason.restype = C.c_char_p
    L.sg_query_count.argtypes = [C.c_void_p]
    L.sg_stream_count.argtypes = [C.c_void_p]
    L.sg_stream_index.argtypes = [C.c_void_p, C.c_char_p]
    L.sg_stream_arity.argtypes = [C.c_void_p, C.c_int]
    return L


def _schema_check(node, schema, defs, path="$"):
    """Minimal draft-07 subset (type, required, enum, const, properties, items, oneOf, $ref) —
    enough to hold the committed descriptors to include/siddhi_gfx_descriptor.schema.json."""
    if "$ref" in schema:
        return _schema_check(node, defs[schema["$ref"].split("/")[-1]], defs, path)
    if "oneOf" in schema:
        ok = [s for s in schema["oneOf"] if not _schema_check(node, s, defs, path)]
        return [] if len(ok) == 1 else [f"{path}: {len(ok)} oneOf branches match"]
    errs = []
    t = schema.get("type")
    tmap = {"object": dict, "array": list, "string": str, "boolean": bool, "integer": int, "null": type(None)}
    if t is not None:
        ts = t if isinstance(t, list) else [t]
        if not any(isinstance(node, tmap[x]) and not (x == "integer" and isinstance(node, bool)) for x in ts):
            return [f"{path}: expected {t}"]
    if "const" in schema and node != schema["const"]:
        errs.append(f"{path}: expected {schema['const']!r}")
    if "enum" in schema and node not in schema["enum"]:
        errs.append(f"{path}: {node!r} not in enum")
    if isinstance(node, dict):
        for r in schema.get("required", []):
            if r not in node:
                errs.append(f"{path}: missing {r}")
        for k, v in node.items():
            if k in schema.get("properties", {}):
                errs += _schema_check(v, schema["properties"][k], defs, f"{path}.{k}")
            elif isinstance(schema.get("additionalProperties"), dict):
                errs += _schema_check(v, schema["additionalProperties"], defs, f"{path}.{k}")
    if isinstance(node, list) and "items" in schema:
        it = schema["items"]
        for i, v in enumerate(node):
            s = it[i] if isinstance(it, list) else it
            if isinstance(it, list) and i >= len(it):
                break
            errs += _schema_check(v, s, defs, f"{path}[{i}]")
    return errs


@pytest.mark.parametrize("name", sorted(EXPECT))
def test_descriptor_matches_schema(name):
    schema = json.load(open(SCHEMA))
    d = json.load(open(os.path.join(DESC, name + ".json")))
    assert _schema_check(d, schema, schema["definitions"]) == []


@pytest.mark.parametrize("name", sorted(EXPECT))
def test_create_app_from_descriptor_without_gpu(L, name):
    raw = open(os.path.join(DESC, name + ".json"), "rb").read()
    h = C.c_void_p()
    rc = L.sg_app_create(raw, None, C.byref(h))
    assert rc == 0, L.sg_last_error()
    try:
        d = json.loads(raw)
        assert L.sg_query_count(h) == len(d["queries"])
        assert L.sg_stream_count(h) == len(d["streams"])
        for q, want in EXPECT[name].items():
            qi = L.sg_query_index(h, q.encode())
            assert qi >= 0
            assert PATH[L.sg_query_path(h, qi)] == want
            reason = L.sg_query_unsupported_reason(h, qi)
            assert (reason is not None) == (want == "unsupported")
        si = L.sg_stream_index(h, b"StockStream")
        assert L.sg_stream_arity(h, si) == 3
        assert L.sg_stream_arity(h, 99) < 0          # bounds-checked, no exception across the ABI
        assert L.sg_query_path(h, 99) < 0
    finally:
        L.sg_app_destroy(h)


def test_descriptor_version_is_checked(L):
    d = json.load(open(os.path.join(DESC, "config1.json")))
    d["version"] = 99
    h = C.c_void_p()
    assert L.sg_app_create(json.dumps(d).encode(), None, C.byref(h)) == -1
    assert b"version" in L.sg_last_error()


def test_every_committed_descriptor_is_covered():
    names = {os.path.basename(p)[:-5] for p in glob.glob(os.path.join(DESC, "*.json"))}
    assert names == set(EXPECT)

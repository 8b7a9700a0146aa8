"""Transcribe known-answer tests from the reference's TestNG suites into JSON fixtures.

Run in the build container (where /root/reference exists):
    python tests/golden/extract_kats.py
It reads the reference test sources *as text* and writes tests/golden/kats_auto.json: per
@Test method the QL string, the InputHandler sends / Thread.sleep timeline, the registered
callbacks and the values the test asserts (assertArrayEquals rows in source order, the final
in/remove event counts).  Only data is written — QL text, input events and expected outputs.
A fixture is kept only if every piece could be transcribed mechanically; tests/golden/kats.json
is the reviewed subset (tests/golden/review_kats.py records per-test decisions).
"""
import json
import os
import re
import sys

REF = "/root/reference/modules/siddhi-core/src/test/java/io/siddhi/core/query/"
FILES = [
    "pattern/WithinPatternTestCase.java",
    "pattern/EveryPatternTestCase.java",
    "pattern/CountPatternTestCase.java",
    "pattern/LogicalPatternTestCase.java",
    "pattern/ComplexPatternTestCase.java",
    "sequence/SequenceTestCase.java",
    "partition/PatternPartitionTestCase.java",
    "partition/SequencePartitionTestCase.java",
    "window/LengthWindowTestCase.java",
    "window/LengthBatchWindowTestCase.java",
    "window/TimeWindowTestCase.java",
    "pattern/absent/AbsentPatternTestCase.java",
    "pattern/absent/EveryAbsentPatternTestCase.java",
    "pattern/absent/LogicalAbsentPatternTestCase.java",
    "pattern/absent/AbsentWithEveryPatternTestCase.java",
    "sequence/absent/AbsentSequenceTestCase.java",
    "sequence/absent/AbsentWithEverySequenceTestCase.java",
    "sequence/absent/EveryAbsentSequenceTestCase.java",
    "sequence/absent/LogicalAbsentSequenceTestCase.java",
    "GroupByTestCase.java",
    "OrderByLimitTestCase.java",
    "partition/WindowPartitionTestCase.java",
]


def java_strings(expr):
    return "".join(m.group(1).replace('\\"', '"').replace("\\n", "\n")
                   for m in re.finditer(r'"((?:[^"\\]|\\.)*)"', expr))


def methods(src):
    for m in re.finditer(r'@Test[^\n]*\n\s*public void (\w+)\(\)[^{]*\{', src):
        start = m.end()
        depth = 1
        i = start
        while depth and i < len(src):
            if src[i] == '{':
                depth += 1
            elif src[i] == '}':
                depth -= 1
            i += 1
        yield m.group(1), src[start:i], src[:m.start()].count('\n') + 1, src[:i].count('\n') + 1


def split_top(s):
    out, depth, cur, q = [], 0, "", None
    for ch in s:
        if q:
            cur += ch
            if ch == q:
                q = None
            continue
        if ch in "\"'":
            q = ch
            cur += ch
            continue
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


class Untranscribable(Exception):
    pass


def int_expr(tok):
    """An integer literal or constant arithmetic (`400 * 3`)."""
    if not re.fullmatch(r"[\d\s*+\-()]+", tok.strip()):
        raise Untranscribable("count expr " + tok)
    return int(eval(tok))


def lit(tok):
    tok = tok.strip()
    if tok == "null":
        return None
    if tok in ("true", "false"):
        return tok == "true"
    m = re.fullmatch(r'"((?:[^"\\]|\\.)*)"', tok)
    if m:
        return m.group(1)
    m = re.fullmatch(r"\(\s*(?:float|double|int|long)\s*\)\s*(.*)", tok)
    if m:
        return lit(m.group(1))
    m = re.fullmatch(r"(-?\d+(?:\.\d*)?(?:[eE][-+]?\d+)?)([fFdDlL]?)", tok)
    if m:
        num, suf = m.groups()
        if suf in ("f", "F"):
            return {"f32": float(num)}
        if suf in ("l", "L"):
            return int(num)
        if suf in ("d", "D") or "." in num or "e" in num.lower():
            return {"f64": float(num)}
        return int(num)
    raise Untranscribable(tok)


def obj_array(expr, clock_value=None):
    """Object[] literal; `clock_value` evaluates the test's clock expressions (`++now`) in Java's
    left-to-right order."""
    m = re.search(r"new Object\[\]\s*\{(.*)\}\s*$", expr.strip(), re.S)
    if not m:
        raise Untranscribable(expr)
    out = []
    for t in split_top(m.group(1)):
        if clock_value is not None and re.fullmatch(r"(\+\+)?[A-Za-z_]\w*(\+\+)?", t.strip()) and t.strip() not in ("null", "true", "false"):
            out.append(clock_value(t))
        else:
            out.append(lit(t))
    return out


def unroll(body):
    """Unroll `for (int i = A; i < B; i++) { ... }` loops whose body does not use the loop variable
    (a repeated send timeline)."""
    while True:
        m = re.search(r"for\s*\(\s*int\s+(\w+)\s*=\s*(\d+)\s*;\s*\1\s*<\s*(\d+)\s*;\s*\1\+\+\s*\)\s*\{", body)
        if not m:
            return body
        depth, i = 1, m.end()
        while depth and i < len(body):
            depth += {"{": 1, "}": -1}.get(body[i], 0)
            i += 1
        inner = body[m.end():i - 1]
        if re.search(r"\b%s\b" % m.group(1), inner):
            return body
        body = body[:m.start()] + inner * (int(m.group(3)) - int(m.group(2))) + body[i:]


def transcribe(path, name, body, line0, line1):
    # int / long constants spliced into QL text (`"lengthBatch(" + length + ")"`)
    consts = {m.group(1): m.group(2) for m in
              re.finditer(r'(?:final\s+)?(?:int|long)\s+(\w+)\s*=\s*(-?\d+)L?\s*;', body)}
    strings = {}

    def concat(expr):
        out = ""
        for tok in re.findall(r'"(?:[^"\\]|\\.)*"|[\w.]+|\S', expr):
            if tok == "+":
                continue
            if tok.startswith('"'):
                out += java_strings(tok)
            elif tok in strings:
                out += strings[tok]
            elif tok in consts:
                out += consts[tok]
            else:
                raise Untranscribable("app expr " + tok)
        return out
    for am in re.finditer(r'String (\w+)\s*=\s*((?:"(?:[^"\\]|\\.)*"|[\w.]+|\s|\+)+);', body, re.S):
        strings[am.group(1)] = concat(am.group(2))
    cm = re.search(r"createSiddhiAppRuntime\(([^;]*)\);", body)
    if not cm:
        raise Untranscribable("no createSiddhiAppRuntime")
    ql = concat(cm.group(1))
    handlers = {}
    for hm in re.finditer(r'InputHandler (\w+)\s*=\s*\w+\.getInputHandler\("(\w+)"\)', body):
        handlers[hm.group(1)] = hm.group(2)
    callbacks = []
    for cbm in re.finditer(r'addCallback\("(\w+)",\s*new (QueryCallback|StreamCallback)', body):
        callbacks.append({"query" if cbm.group(2) == "QueryCallback" else "stream": cbm.group(1)})
    ops = []
    expect_rows = []
    counts = {}
    body = unroll(body)
    if re.search(r"\b(for|while)\s*\([^)]*\)\s*\{[^}]*\.send\(", body, re.S):
        raise Untranscribable("send inside a loop")
    clock = {}

    def ts_value(tsx):
        tsx = tsx.strip()
        m = re.fullmatch(r"(\+\+)?(\w+)(\+\+)?(?:\s*([-+])\s*(\d+)L?)?", tsx)
        if m and m.group(2) in clock:
            var = m.group(2)
            if m.group(1):
                clock[var] += 1
            v = clock[var]
            if m.group(3):
                clock[var] += 1
            if m.group(4):
                v = v + int(m.group(5)) if m.group(4) == "+" else v - int(m.group(5))
            return v
        if re.fullmatch(r"-?\d+L?", tsx):
            return int(tsx.rstrip("L"))
        raise Untranscribable("ts expr " + tsx)

    # callback bodies: assertEquals there checks each delivered event against the callback's own counters
    # (not the final counts); those are transcribed by hand (review_kats.py MANUAL)
    spans = []
    for rm in re.finditer(r"public void receive\([^)]*\)\s*\{", body):
        depth, i = 1, rm.end()
        while depth and i < len(body):
            depth += {"{": 1, "}": -1}.get(body[i], 0)
            i += 1
        spans.append((rm.end(), i))
    in_cb = 0
    for sm in re.finditer(r'(\w+)\.send\(([^;]*)\);|Thread\.sleep\((\d+)\)|(assert\w*)\(([^;]*)\);|long (\w+)\s*=\s*([^;]+);|(\w+)\s*\+=\s*([^;]+);', body, re.S):
        if sm.group(6):
            rhs = sm.group(7).strip()
            if rhs == "System.currentTimeMillis()":
                clock[sm.group(6)] = 1_600_000_000_000
            elif re.fullmatch(r"-?\d+L?", rhs):
                clock[sm.group(6)] = int(rhs.rstrip("L"))
            continue
        if sm.group(8):
            if sm.group(8) in clock:
                expr = sm.group(9).split("//")[0].replace("L", "")
                if not re.fullmatch(r"[\d\s*+\-()]+", expr):
                    raise Untranscribable("clock expr " + expr)
                clock[sm.group(8)] += int(eval(expr))
            continue
        if sm.group(1):
            var, args = sm.group(1), sm.group(2)
            if var not in handlers:
                raise Untranscribable("send on " + var)
            a = split_top(args)
            if len(a) == 1 and re.match(r"new Event\[\]\s*\{", a[0].strip()):
                inner = a[0].strip()[a[0].index("{") + 1:a[0].rindex("}")]
                evs = []
                for ev in split_top(inner):
                    em = re.fullmatch(r"new Event\((.*)\)", ev.strip(), re.S)
                    if not em:
                        raise Untranscribable("event form " + ev[:40])
                    ea = split_top(em.group(1))
                    evs.append([ts_value(ea[0]), obj_array(ea[1], ts_value)])
                ops.append(["send_batch", handlers[var], evs])
            elif len(a) == 1 and "new Object[]" in a[0]:
                ops.append(["send", handlers[var], None, obj_array(a[0], ts_value)])
            elif len(a) == 2 and "new Object[]" in a[1]:
                ts = ts_value(a[0])
                ops.append(["send", handlers[var], ts, obj_array(a[1], ts_value)])
            else:
                raise Untranscribable("send form " + args[:60])
        elif sm.group(3):
            ops.append(["sleep", int(sm.group(3))])
        elif sm.group(4):
            fn, args = sm.group(4), sm.group(5)
            if fn == "assertArrayEquals" and "new Object[]" in args:
                first = split_top(args)[0]
                expect_rows.append(obj_array(first))
            elif fn in ("assertEquals", "assertTrue", "assertFalse") and any(a0 <= sm.start() < a1 for a0, a1 in spans):
                in_cb += 1
            elif fn == "assertEquals":
                a = split_top(args)
                if len(a) == 3 and "inEventCount" in a[2]:
                    counts["in_count"] = int_expr(a[1])
                elif len(a) == 3 and "removeEventCount" in a[2]:
                    counts["rm_count"] = int_expr(a[1])
                elif len(a) == 2 and "inEventCount" in a[1] and re.fullmatch(r"\d+", a[0]):
                    counts["in_count"] = int(a[0])
                elif len(a) == 3 and "eventArrived" in a[2]:
                    counts["arrived"] = a[1] == "true"
            elif fn == "assertTrue" or fn == "assertFalse":
                pass
        elif sm.group(6):
            pass
    return {
        "name": f"{os.path.basename(path)[:-5]}.{name}",
        "source": f"TEST/query/{path}:{line0}-{line1}",
        "app": ql,
        "callbacks": callbacks,
        "ops": ops,
        "expect": {"rows": expect_rows, **counts},
        "in_callback_asserts": in_cb,
    }


def main():
    out = []
    skipped = []
    for f in FILES:
        src = open(REF + f).read()
        for name, body, l0, l1 in methods(src):
            try:
                out.append(transcribe(f, name, body, l0, l1))
            except Untranscribable as e:
                skipped.append((f, name, str(e)[:80]))
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats_auto.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(f"transcribed {len(out)}; skipped {len(skipped)}")
    for s in skipped:
        print("  skip", *s)


if __name__ == "__main__":
    main()

"""Dump the structure of reference TestNG cases (study aid; reads reference test sources as text).

For each @Test method prints: the concatenated QL strings, the sequence of InputHandler
sends / Thread.sleep calls, and the assertion lines. Used to transcribe known-answer
fixtures into tests/golden/ by hand.
"""
import re, sys

def java_strings(expr):
    return "".join(m.group(1) for m in re.finditer(r'"((?:[^"\\]|\\.)*)"', expr))

def methods(src):
    for m in re.finditer(r'@Test[^\n]*\n\s*public void (\w+)\(\)[^{]*\{', src):
        start = m.end(); depth = 1; i = start
        while depth and i < len(src):
            if src[i] == '{': depth += 1
            elif src[i] == '}': depth -= 1
            i += 1
        yield m.group(1), src[start:i], src[:m.start()].count('\n') + 1

def main(path, only=None):
    src = open(path).read()
    for name, body, line in methods(src):
        if only and name not in only: continue
        print(f"## {name}  (line {line})")
        assigns = {}
        for am in re.finditer(r'String (\w+)\s*=\s*((?:"[^\n]*"\s*\+?\s*)+);', body, re.S):
            assigns[am.group(1)] = java_strings(am.group(2))
        for k, v in assigns.items():
            print(f"  {k}: {v}")
        for sm in re.finditer(r'(\w+)\.send\(([^;]*)\);|Thread\.sleep\((\d+)\)|(assert\w*\([^;]*\));', body):
            if sm.group(1): print(f"  SEND {sm.group(1)} {sm.group(2)}")
            elif sm.group(3): print(f"  SLEEP {sm.group(3)}")
            else: print(f"  {sm.group(4)}")

if __name__ == "__main__":
    main(sys.argv[1], set(sys.argv[2:]) or None)

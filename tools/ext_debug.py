"""Drive one extension window through per-event chunks and print its chunks (debugging aid for ext.hip)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import test_ext_cpu as cpu  # noqa: E402

if __name__ == "__main__":
    import torch
    torch.cuda.init()
    L = cpu.load_lib()
    w = cpu.Window(L, "time", 2000)
    d = cpu._stream(20, 7)
    for i in range(len(d["ts"])):
        t = int(d["ts"][i])
        w.on_time(t)
        w.process([i], [t], t)
        print(i, t, [(list(a), list(b)) for a, b, _ in w.chunks()], flush=True)

"""Summarise a rocprofv3 --kernel-trace --stats run (rocpd SQLite output) as a small CSV.

    python tools/prof_summary.py gpurun_out/prof_TAG/prof_results.db > profiles/rNN_TAG_kernel_stats.csv
"""
import re
import sqlite3
import sys


def short(name: str) -> str:
    if "rocprim" in name:
        m = re.search(r"detail::(\w+?)(?:_config|<)", name)
        return "rocprim::" + (m.group(1) if m else "kernel")
    return re.sub(r"\(.*$", "", name)[:120]


def main(db: str) -> None:
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    print("kernel,calls,total_us,avg_us,percent")
    for name, calls, tot, avg, pct in rows:
        print(f"\"{short(name)}\",{calls},{tot:.3f},{avg:.3f},{pct:.2f}")


if __name__ == "__main__":
    main(sys.argv[1])

"""Summarise a rocprofv3 --kernel-trace --stats database (rocpd sqlite) as a markdown table.

    python tools/prof_summary.py gpurun_out/prof2/run_results.db [--top 30] [--match SUBSTR]
Durations in the db are microseconds; the table reports calls, total ms, average us and share.
"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name) if not name.startswith("void cdm::gemm") else name.split("(")[0]
    return name.replace("void ", "").replace("cdm::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--match", default=None)
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = list(cur.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    if a.match:
        rows = [r for r in rows if a.match in r[0]]
    tot = sum(r[2] for r in rows)
    print(f"| kernel | calls | total ms | avg us | % |\n|---|---:|---:|---:|---:|")
    for name, calls, total, avg, pct in rows[: a.top]:
        print(f"| `{short(name)}` | {calls} | {total/1e3:.3f} | {avg:.1f} | {100*total/tot:.1f} |")
    print(f"\n_total kernel time {tot/1e3:.1f} ms over {sum(r[1] for r in rows)} dispatches_")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""The mixed path's fixed cost before the hash, from a rocprofv3 kernel
trace (SQLite, rocprofv3 --kernel-trace -d DIR): for every mixed-kernel
dispatch, the sort, layout and planner kernels enqueued before it on the
same stream since the previous hash kernel -- each one's duration and the
span from the first one's start to the mixed kernel's start (launch gaps
included).  Usage: python tools/fixed_cost.py DIR/run_results.db [...]"""
import json
import sqlite3
import sys

PRE = ("sort_keys_hist", "sort_hist", "sort_scatter", "hist_scan", "plan_layout_tail_kernel", "plan_layout_kernel",
       "plan_mixed_kernel", "block_keys16", "gather_lengths", "rocprim")


def short(name):
    for p in PRE + ("sha1_mixed",):
        if p in name:
            if p in ("sort_scatter", "sort_hist"):
                return p + ("<1>" if ("<1>" in name or "ILi1E" in name) else "<2>")
            return p
    return None


def main():
    for db in sys.argv[1:]:
        c = sqlite3.connect(db)
        rows = c.execute("select name, start, end, grid_x from kernels order by start").fetchall()
        pend, out = [], []
        for name, s, e, gx in rows:
            k = short(name)
            if k is None:
                pend = []
                continue
            if k == "sha1_mixed":
                if pend:
                    per = {}
                    for kk, ss, ee in pend:
                        per[kk] = round(per.get(kk, 0) + (ee - ss) / 1e3, 2)
                    out.append({"kernels_us": per, "sum_us": round(sum(per.values()), 2),
                                "span_to_hash_start_us": round((s - pend[0][1]) / 1e3, 2),
                                "hash_ms": round((e - s) / 1e6, 3)})
                pend = []
            else:
                pend.append((k, s, e))
        for r in out:
            print(json.dumps(dict(db=db, **r)))


if __name__ == "__main__":
    main()

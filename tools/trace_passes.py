#!/usr/bin/env python3
"""Per-pass timeline of a bucket-range-pass build from a rocprofv3
--kernel-trace CSV: for every pass (a k_sel<1> launch starts one) the main
solve's (k_gov_solve) and the oversized-bucket solve's (k_gov_solve_big) start
and end, in ms from the first kernel, and which one ended last.

    python tools/trace_passes.py <..._kernel_trace.csv> [--json out.json]
"""
import csv
import json
import sys


def main():
    path = sys.argv[1]
    rows = []
    import gzip
    with (gzip.open(path, "rt") if path.endswith(".gz") else open(path)) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    t0 = rows[0][0]
    ms = lambda t: (t - t0) / 1e6  # noqa: E731
    passes = []
    cur = None
    for s, e, name in rows:
        short = name.split("(")[0].split("<")[0].replace("void ", "").strip().split("::")[-1]
        if short == "k_sel" and "<1" in name:
            cur = {"sel_start": ms(s), "kernels": {}}
            passes.append(cur)
        if cur is None:
            continue
        k = cur["kernels"].setdefault(short, {"start": ms(s), "end": ms(e), "launches": 0, "busy_ms": 0.0})
        k["start"] = min(k["start"], ms(s))
        k["end"] = max(k["end"], ms(e))
        k["launches"] += 1
        k["busy_ms"] += (e - s) / 1e6
    out = []
    for i, p in enumerate(passes):
        kk = p["kernels"]
        main_k = kk.get("k_gov_solve")
        big_k = kk.get("k_gov_solve_big") or kk.get("k_gov_solve_mid")
        row = {"pass": i, "sel_start_ms": round(p["sel_start"], 2)}
        if main_k:
            row["solve_ms"] = [round(main_k["start"], 2), round(main_k["end"], 2)]
        if big_k:
            row["solve_big_ms"] = [round(big_k["start"], 2), round(big_k["end"], 2)]
            row["big_is_tail"] = bool(main_k and big_k["end"] > main_k["end"])
            row["big_tail_ms"] = round(max(0.0, big_k["end"] - (main_k["end"] if main_k else big_k["start"])), 2)
        row["busy_ms"] = {k: round(v["busy_ms"], 2) for k, v in sorted(kk.items(), key=lambda x: -x[1]["busy_ms"])[:8]}
        out.append(row)
        print(json.dumps(row))
    if len(sys.argv) > 3 and sys.argv[2] == "--json":
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()

"""Per-launch HBM traffic of the pass-1 kernel (k_pass1_d13e) from separate rocprofv3 --pmc passes.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the
bytes of a wide coalesced streaming read -> x2; WRITE_SIZE is exact for
16-B/lane streams (the 16-B id-run stores).  Units KiB.
usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON"""
import csv, json, sys

def per_dispatch(path, counter, kernel="k_pass1_d13"):  # matches k_pass1_d13e too
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
            vals[int(r["Dispatch_Id"])] = float(r["Counter_Value"]) * 1024
    return [vals[k] for k in sorted(vals)]

fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
write = per_dispatch(sys.argv[2], "WRITE_SIZE")
n = 13_193_787_549
launches = len(fetch)
out = {
    "kernel": "k_pass1_d13e (the bench's pass-1 launches)",
    "launches_per_step": launches,
    "keys_per_launch": n / launches,
    "read_bytes_per_launch": 2 * sum(fetch) / launches,
    "write_bytes_per_launch": sum(write) / len(write),
    "hbm_bytes_per_launch": 2 * sum(fetch) / launches + sum(write) / len(write),
    "algorithmic_read_bytes_per_launch": 13 * n / launches,
    "note": "FETCH_SIZE x2 (gfx950 streaming-read under-count) + WRITE_SIZE, KiB units; one --pmc counter per pass",
}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out))

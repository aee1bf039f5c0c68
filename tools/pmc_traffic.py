"""Per-launch HBM traffic of the pass-1 kernel (k_pass1_d13e) from separate rocprofv3 --pmc passes.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the
bytes of a wide coalesced streaming read -> x2; WRITE_SIZE is exact for
16-B/lane streams (the 16-B id-run stores).  Units KiB.
The output names the library the counters were collected with (its sha256):
bench.py reports this traffic only for that same library.
usage: python tools/pmc_traffic.py FETCH_CSV WRITE_CSV OUT_JSON [ROUND]"""
import csv, hashlib, json, os, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()

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
    "round": int(sys.argv[4]) if len(sys.argv) > 4 else None,
    "library_sha256": sha256(os.environ.get("BSDB_LIB") or os.path.join(ROOT, "bsdb_amd", "libbsdb_mi355x.so")),
    "source": "tools/gpu_pmc_bench.sh (rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE, over bench.py --steps 1)",
}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out))

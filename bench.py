#!/usr/bin/env python3
"""bench.py -- device-resident index-build keys/s on MI355X (BASELINE.json metric).

One step = the hot path over the whole synthetic key set that is resident in
HBM: SpookyHash-short per key -> GOV bucket -> bucket-occupancy histogram
(two-pass partitioned kernels) -> [N>1: RCCL all-reduce of the histogram over
xGMI] -> edge offsets E[] (the low 56 bits of edgeOffsetAndSeed).

Workload (default): BASELINE.json config 4, the README dataset shape,
n = 13 193 787 549 keys x 13 bytes (171.5 GB), exact index, hash.checksum.bits=4,
m = n/1500+1 = 8 795 859 buckets.  It fits one MI355X, so N=1 runs the whole
set; with --gpus N the same key set is sharded N ways (strong scaling).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n KEYS] [--no-cpu]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from bsdb_amd.distributed import shard  # noqa: E402

README_N = 13_193_787_549     # README.md:50-60 record count
KEY_LEN = 13
HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md chip table: 8.0 TB/s HBM3E



def _lib_sha256():
    """sha256 of the HIP library this process loads (BSDB_LIB or the in-tree build)."""
    import hashlib
    path = os.environ.get("BSDB_LIB") or os.path.join(ROOT, "bsdb_amd", "libbsdb_mi355x.so")
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    return O


def cpu_baseline(m: int, target_s: float, threads: int):
    """The oracle's multi-threaded hash+bucket+histogram on resident 13-byte keys
    (same key recipe, same m), timed on this box's host cores; bounded sample."""
    O = _oracle()
    calib_n = 4_000_000
    keys = O.gen_keys13_mt(0, calib_n, threads)
    _, dt = O.histogram_fixed_mt(keys, KEY_LEN, m, threads)
    rate = calib_n / max(dt, 1e-6)
    n = int(min(max(rate * target_s, calib_n), 400_000_000))
    keys = O.gen_keys13_mt(0, n, threads)
    total_keys, total_s = 0, 0.0
    passes = 0
    while total_s < target_s * 0.9 or passes == 0:
        _, dt = O.histogram_fixed_mt(keys, KEY_LEN, m, threads)
        total_keys += n
        total_s += dt
        passes += 1
        if passes >= 8:
            break
    del keys
    return {"value": total_keys / total_s, "unit": "keys/s", "cores": threads, "kind": "port",
            "cpu_model": O.cpu_model(), "os_cpu_count": os.cpu_count(),
            "sample": f"{passes} pass(es) over {n} resident 13-byte keys (first {n} of the workload's key recipe), "
                      f"m={m}, {total_s:.1f} s of CPU work, {threads} threads (every CPU this process may use: "
                      f"affinity capped by the cgroup quota; os.cpu_count() = {os.cpu_count()} counts the whole "
                      f"machine), oracle bo_histogram_fixed_mt (C restatement pinned to the reference's spooky.c)"}


def full_build_gpu(ctx, n: int, width: int, reps: int):
    """Full build on the device, keys resident in HBM: hash -> GOV build
    (bucket sort, per-bucket solve that also signs with `width` checksum bits
    and returns every key's rank, F2) -> index scatter of the record
    addresses (W:129-145).  keys/s over the median run, per-stage device time."""
    import torch
    keys = ctx.gen_keys13(0, n)
    addr = torch.arange(n, dtype=torch.int64, device="cuda")
    index = torch.empty(n, dtype=torch.int64, device="cuda")
    runs = []
    for _ in range(reps + 1):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        sig = ctx.hash_fixed(keys, 13)
        ev[1].record()
        E, vals, sb, rank = ctx.gov_build_ranks(sig, width)
        ev[2].record()
        ctx.index_scatter(rank, addr, 0, n, index)
        ev[3].record()
        torch.cuda.synchronize()
        runs.append([ev[i].elapsed_time(ev[i + 1]) for i in range(3)])
        del sig, E, vals, sb, rank
    runs = sorted(runs[1:], key=sum)
    hash_ms, gov_ms, index_ms = runs[len(runs) // 2]
    total = hash_ms + gov_ms + index_ms
    del keys, addr, index
    torch.cuda.empty_cache()
    return {"n_keys": n, "checksum_bits": width, "keys_per_s": n / (total / 1e3), "ms": total,
            "stage_ms": {"hash": hash_ms, "gov_build_sort_solve_sign_rank": gov_ms, "index_scatter": index_ms}}


def e2e_host_to_disk(ctx, n: int, width: int):
    """Keys in host memory -> hash.dump + index.db on disk through the host ABI
    (bsdb_mph_build_index_fixed: hash, GOV build with ranks, index scatter,
    <= 128 MiB writes; then bsdb_mph_dump), PCIe and file writes included.
    Keys generated on the device and copied to host memory before timing."""
    import shutil
    import tempfile
    import time as _t
    import numpy as np
    keys = ctx.gen_keys13(0, n)[: 13 * n].cpu().numpy()
    addr = np.uint64(0x1000) + np.uint64(48) * np.arange(n, dtype=np.uint64)  # SimpleCompact 48-B records
    d = tempfile.mkdtemp(prefix="bsdb_e2e_", dir="/tmp")
    try:
        t0 = _t.perf_counter()
        mph = ctx.mph_build_index_fixed(keys, 13, width, addr, os.path.join(d, "index.db"),
                                        os.path.join(d, "index_a.db"))
        mph.dump(os.path.join(d, "hash.dump"))
        dt = _t.perf_counter() - t0
        size = os.path.getsize(os.path.join(d, "index.db"))
        mph.close()
    finally:
        shutil.rmtree(d, ignore_errors=True)
    assert size == 8 * n
    return {"n_keys": n, "checksum_bits": width, "keys_per_s": n / dt, "ms": dt * 1e3,
            "path": "host keys -> bsdb_mph_build_index_fixed (F2) -> index.db + hash.dump in /tmp"}


def e4_multi_device(ctx, n: int, width: int, ndev: int):
    """E4 in one process over `ndev` GPUs (--e4-devices; bsdb_multi_mph_build_index_fixed
    with no index path: hash of input-order shards -> owner partition -> one
    device-to-device exchange -> range solves -> the MPHF fields in host
    memory), keys in host memory when the clock starts.  With one device it
    is the one-device build through the multi-device entry point.  Both calls
    are reported: the first (cold: it also grows every context's workspace)
    and the second."""
    import time as _t
    import torch
    from bsdb_amd.native import Multi
    keys = ctx.gen_keys13(0, n)[: 13 * n].cpu().numpy()
    torch.cuda.empty_cache()
    times = []
    with Multi(ndev) as mc:
        for _ in range(2):
            t0 = _t.perf_counter()
            E, _, _ = mc.mph_build_index_fixed(keys, 13, width)
            times.append(_t.perf_counter() - t0)
            assert int(E[-1]) & ((1 << 56) - 1) == n
    return {"n_keys": n, "checksum_bits": width, "devices": ndev, "keys_per_s": n / times[1], "ms": times[1] * 1e3,
            "cold_keys_per_s": n / times[0], "cold_ms": times[0] * 1e3,
            "path": f"host keys -> bsdb_multi_mph_build_index_fixed (E4, one process, {ndev} GPU(s)) -> "
                    "E / values / checksum words in host memory"}


def c4_exact_passes(ctx, keys, n: int, width: int):
    """BASELINE C4's exact index on this one GPU, from the headline's resident
    keys (bsdb_dev_mph_build_index_passes_fixed): sequential bucket-range
    passes, each re-hashing every key, sorting, solving and signing its range
    and writing its index.db slots from the solve; each pass's slots are
    copied to host memory while the next pass runs.  Clock: keys in HBM ->
    the GOV structure in HBM + all n index slots in host memory.  One call
    (it also grows the context's workspace)."""
    import time as _t
    import numpy as np
    import torch
    index = np.empty(n, np.uint64)                # index.db, 8 n bytes of host memory
    torch.cuda.synchronize()
    t0 = _t.perf_counter()
    E, vals, sb, used = ctx.mph_build_index_passes(keys, 13, n, width, 0, addr_base=0x1000, addr_stride=48,
                                                   index=index)
    torch.cuda.synchronize()
    dt = _t.perf_counter() - t0
    ok = int(E[-1].item()) & ((1 << 56) - 1) == n
    del E, vals, sb, index
    torch.cuda.empty_cache()
    return {"n_keys": n, "checksum_bits": width, "passes": used, "keys_per_s": n / dt, "ms": dt * 1e3,
            "check": {"E[m]==n": ok},
            "path": "keys resident in HBM -> bsdb_dev_mph_build_index_passes_fixed (per pass: re-hash + range "
                    "select, bucket sort, solve + sign + index slots) -> GOV structure in HBM, index.db slots "
                    "(8 B x n, byte-reversed addr = 0x1000 + 48 i) in host memory"}


def e4_ranks_full_build(ctx, world: int, rank: int, backend: str, width: int, reps: int, n_total: int):
    """The N > 1 full build, one rank per GPU: each rank
    holds its contiguous key shard of n_total keys in HBM (13 B each, the
    headline's recipe) and the timed region is the product's whole build --
    hash the shard, group (sig0, sig1, addr) by bucket-range owner, ONE
    all-to-all, the range build (sort, solve, sign, ranks) into O(n/G) windows,
    each rank's index.db slots placed from its ranks and copied to host
    memory, every window sent to rank 0, which assembles E / values /
    checksum words (distributed.sharded_full_build).  n_total defaults to C4's
    per-GPU share at 8 GPUs times N (C4 itself at N = 8; weak scaling): C4's
    whole key set on fewer GPUs exceeds one GPU's HBM without passes.  Returns
    the max over ranks of each rep's wall time (barrier on both sides)."""
    import time as _t
    import numpy as np
    import torch
    import torch.distributed as dist
    from bsdb_amd.distributed import DeviceBuild, sharded_full_build
    lo, hi = shard(n_total, rank, world)
    nloc = hi - lo
    keys = ctx.gen_keys13(lo, nloc)
    addr = torch.arange(lo, hi, dtype=torch.int64, device="cuda") * 48 + 0x1000  # SimpleCompact 48-B records
    host_index = None
    times, stage = [], None
    red_dev = "cuda" if backend == "nccl" else "cpu"
    for rep in range(reps + 1):  # rep 0 warms the workspace and the allocator
        torch.cuda.synchronize()
        dist.barrier()
        t0 = _t.perf_counter()
        sig = ctx.hash_fixed(keys[: 13 * nloc], 13)
        torch.cuda.synchronize()
        t1 = _t.perf_counter()
        res = sharded_full_build(DeviceBuild(ctx), sig, addr, n_total, width)
        del sig
        torch.cuda.synchronize()
        t2 = _t.perf_counter()
        idx = res["index"]
        if host_index is None or host_index.numel() < idx.numel():
            host_index = torch.empty(idx.numel(), dtype=torch.int64)
        host_index[: idx.numel()].copy_(idx)  # index.db slots of this rank's range, in host memory
        t3 = _t.perf_counter()
        dist.barrier()
        t4 = _t.perf_counter()
        local = torch.tensor([t4 - t0, t1 - t0, t2 - t1, t3 - t2], dtype=torch.float64, device=red_dev)
        dist.all_reduce(local, op=dist.ReduceOp.MAX)
        if rep:
            times.append(local.tolist())
        ok = rank != 0 or int(res["E"][-1].item()) & ((1 << 56) - 1) == n_total
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=red_dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        sent = torch.tensor([res["bytes_sent"]], dtype=torch.float64, device=red_dev)
        dist.all_reduce(sent, op=dist.ReduceOp.MAX)
        del res, idx
    del keys, addr, host_index
    torch.cuda.empty_cache()
    ctx.release_workspace()
    best = min(times, key=lambda t: t[0])
    return {"n_keys": n_total, "checksum_bits": width, "ranks": world, "keys_per_s": n_total / best[0],
            "ms": best[0] * 1e3, "reps": reps,
            "stage_ms_max_over_ranks": {"hash": best[1] * 1e3, "exchange_build_assemble": best[2] * 1e3,
                                        "index_d2h": best[3] * 1e3},
            "max_bytes_sent_per_rank": float(sent.item()), "check": {"E[m]==n": bool(flag.item())},
            "scaling": "weak (C4/8 keys per GPU; C4 at N = 8)",
            "path": "per rank: shard keys in HBM -> hash -> owner partition -> ONE all-to-all of (sig0, sig1, addr) "
                    "-> bsdb_dev_gov_build_window (sort, solve, sign, ranks) -> index slots to host memory; "
                    "windows to rank 0 (point to point), which ORs them into the GOV structure"}


def _roomiest_dir(need_bytes: float):
    """The candidate directory with the most free space, or None when none has
    room for `need_bytes` (the figure then writes to /dev/null and says so)."""
    import shutil
    best, free = None, -1
    for d in ("/tmp", "/dev/shm", os.path.join(ROOT, "build")):
        try:
            os.makedirs(d, exist_ok=True)
            f = shutil.disk_usage(d).free
        except OSError:
            continue
        if f > free:
            best, free = d, f
    return (best, free) if free > need_bytes * 1.1 else (None, free)


def e2e_c4_host_passes(ctx, n: int, width: int, chunk: int = 1 << 28):
    """BASELINE C4 from HOST memory on one GPU (bsdb_builder_*, what the JVM
    calls): the 13.19e9 keys arrive in host batches of `chunk` keys (each
    batch is produced before the clock runs for it: generated on the device
    and copied to a pinned host buffer), every add() copies its batch into
    HBM, then finish() runs the bucket-range passes and writes index.db at
    each pass's offset while the next pass solves.  Timed: the adds + the
    finish (host keys -> index.db on disk + the MPHF in HBM); record
    addresses 0x1000 + 48 i (fixed 48-byte records of one file)."""
    import shutil
    import tempfile
    import time as _t
    import torch
    d, free = _roomiest_dir(8 * n)
    tmp = tempfile.mkdtemp(prefix="bsdb_c4_", dir=d) if d else None
    ip = os.path.join(tmp, "index.db") if tmp else "/dev/null"
    try:
        dev = torch.empty(13 * chunk + 16, dtype=torch.uint8, device="cuda")
        host = torch.empty(13 * chunk, dtype=torch.uint8, pin_memory=True)
        b = ctx.builder(13, key_capacity=n, addr_base=0x1000, addr_stride=48)
        t_add = 0.0
        for k0 in range(0, n, chunk):
            k = min(chunk, n - k0)
            ctx.gen_keys13(k0, k, out=dev)
            host[: 13 * k].copy_(dev[: 13 * k])
            torch.cuda.synchronize()
            t0 = _t.perf_counter()
            b.add_fixed(host[: 13 * k].numpy(), 13)
            t_add += _t.perf_counter() - t0
        del dev
        torch.cuda.empty_cache()
        t0 = _t.perf_counter()
        mph, used = b.finish(width, ip, None)
        t_fin = _t.perf_counter() - t0
        size = os.path.getsize(ip) if tmp else None
        E, _, _ = mph.export()
        ok = int(E[-1]) & ((1 << 56) - 1) == n
        mph.close()
        b.close()
        del host
    finally:
        if tmp:
            shutil.rmtree(tmp, ignore_errors=True)
    dt = t_add + t_fin
    return {"n_keys": n, "checksum_bits": width, "passes": used, "keys_per_s": n / dt, "ms": dt * 1e3,
            "add_ms": t_add * 1e3, "finish_ms": t_fin * 1e3, "h2d_GBps": 13 * n / t_add / 1e9,
            "index_db": ip if tmp is None else f"{d} ({size} bytes; {free / 1e9:.0f} GB free before)",
            "check": {"E[m]==n": ok, "index.db bytes == 8n": (size == 8 * n) if tmp else None},
            "path": "host keys (batches of 2^28) -> bsdb_builder_add_fixed (H2D into HBM) -> bsdb_builder_finish "
                    "(bucket-range passes; each pass's index.db slots pwritten at their offset while the next "
                    "pass solves) -> index.db" + ("" if tmp else " written to /dev/null: no file system on this "
                                                  "box had room for 8n bytes")}


def usable_cpus() -> int:
    """CPUs this process may use: the affinity mask capped by the cgroup quota
    (the GPU box's os.cpu_count() counts the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return max(1, n)


def e2e_kv_to_disk(ctx, n: int, width: int, partitions: int = 8, approximate: bool = False, threads: int = 0):
    """BASELINE C2 / C3 from the DATA FILES: n records of 13-byte keys and
    32-byte values in SimpleCompactKVWriter's layout (48-byte records,
    kv.db.<p>, written before the clock) -> bsdb_kv_build_index (host threads
    parse the partitions and stream them into the builder; bucket-range-pass
    build; index.db, and index_a.db's value slots in approximate mode) +
    hash.dump.  The reference's buildIndex reads the same files (W:134,
    PartitionedKVWriter.java:50-70), which its writer splits into
    2 x availableProcessors() partitions (PartitionedKVWriter.java:14)."""
    import shutil
    import tempfile
    import time as _t
    import torch
    need = 48 * n + 8 * n * (2 if approximate else 1)
    d, _ = _roomiest_dir(need)
    if d is None:
        return {"skipped": f"no directory with {need / 1e9:.1f} GB free"}
    tmp = tempfile.mkdtemp(prefix="bsdb_kv_", dir=d)
    try:
        base = os.path.join(tmp, "kv.db")
        per = -(-n // partitions)
        for p in range(partitions):
            lo, hi = p * per, min(n, (p + 1) * per)
            with open(f"{base}.{p}", "wb") as f:
                for c0 in range(lo, hi, 1 << 24):
                    k = min(1 << 24, hi - c0)
                    rec = torch.empty((k, 48), dtype=torch.uint8, device="cuda")
                    rec[:, 0] = 13
                    rec[:, 1] = 0
                    rec[:, 2] = 32
                    rec[:, 3:16] = ctx.gen_keys13(c0, k).view(k, 13)
                    rec[:, 16:] = torch.randint(0, 256, (k, 32), dtype=torch.uint8, device="cuda")
                    rec.cpu().numpy().tofile(f)
                    del rec
        torch.cuda.empty_cache()
        ip, ap = os.path.join(tmp, "index.db"), os.path.join(tmp, "index_a.db")
        t0 = _t.perf_counter()
        mph = ctx.kv_build_index(base, partitions, width, ip, ap, approximate=approximate, threads=threads)
        mph.dump(os.path.join(tmp, "hash.dump"))
        dt = _t.perf_counter() - t0
        size, asize = os.path.getsize(ip), os.path.getsize(ap)
        E, _, _ = mph.export()
        ok = int(E[-1]) & ((1 << 56) - 1) == n
        mph.close()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return {"n_keys": n, "checksum_bits": width, "partitions": partitions, "approximate": approximate,
            "keys_per_s": n / dt, "ms": dt * 1e3, "kv_db_bytes": 48 * n, "host_cpus": usable_cpus(),
            "check": {"E[m]==n": ok, "index.db bytes == 8n": size == 8 * n,
                      "index_a.db bytes": asize == (8 * n if approximate else 0)},
            "path": f"kv.db.<p> files ({48 * n / 1e9:.1f} GB, compact layout, {partitions} partitions, in {d}) -> "
                    "bsdb_kv_build_index (parallel partition scan streamed into the builder, bucket-range-pass "
                    "build) -> index.db" + (" + index_a.db" if approximate else "") + " + hash.dump"}


def single_pass_ab(ctx, keys, n: int, m: int, ref_counts, reps: int = 3):
    """The single-pass histogram (mode 3) on the same resident
    keys: its counts against the headline's, and its time (HIP events).  Opt-in
    design kept for the A/B; the headline is the two-pass path."""
    import torch
    ctx.set_histogram_mode(3)
    try:
        counts = torch.zeros(m, dtype=torch.int32, device="cuda")
        ctx.histogram_fixed(keys, KEY_LEN, m, counts=counts, n=n)
        torch.cuda.synchronize()
        equal = bool(torch.equal(counts, ref_counts))
        launches0 = ctx.fused_status()[0]
        times = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            counts.zero_()
            a.record()
            ctx.histogram_fixed(keys, KEY_LEN, m, counts=counts, n=n)
            b.record()
            torch.cuda.synchronize()
            times.append(a.elapsed_time(b))
        launches, timeouts = ctx.fused_status()
        del counts
    finally:
        ctx.set_histogram_mode(0)
    ms = min(times)
    return {"n_keys": n, "ms": ms, "keys_per_s": n / ms * 1e3, "equal_to_two_pass": equal,
            "single_pass_launches": launches - launches0, "timeouts": timeouts,
            "path": "k_hist13_fused (bucket owners per CU, ids through an on-die ring) + the two-pass path "
                    "for the tail; not the headline"}


def c5_varlen_histogram(ctx, n: int, steps: int):
    """BASELINE C5 shape at its full size on one GPU: 4e9 variable-length keys
    (8-64 B, Zipf, mean ~17.7 B) resident with u64
    offsets, the same hash -> bucket -> histogram -> edge offsets step
    (algorithmic bytes per key = key bytes + the 8-byte offset); then the
    whole build of the same keys (cb = 16) by bucket-range passes."""
    import torch
    blob, off = ctx.gen_keys_var(0, n)
    m = n // 1500 + 1
    counts = torch.zeros(m, dtype=torch.int32, device="cuda")
    E = torch.empty(m + 1, dtype=torch.int64, device="cuda")
    for _ in range(2):
        counts.zero_()
        ctx.histogram_var(blob, off, m, counts=counts)
        ctx.edge_offsets(counts, out=E)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        counts.zero_()
        ctx.histogram_var(blob, off, m, counts=counts)
        ctx.edge_offsets(counts, out=E)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    nbytes = int(off[-1].item()) + 8 * n
    ok = int(E[-1].item()) == n
    del counts, E
    torch.cuda.empty_cache()
    hist = {"n_keys": n, "keys_per_s": n / dt, "ms_per_step": dt * 1e3, "steps": steps,
            "bytes_per_key": nbytes / n, "roofline_frac": nbytes / dt / (HBM_PEAK_GBS * 1e9),
            "check": {"E[m]==n": ok},
            "path": "var-len keys + u64 offsets resident in HBM -> histogram (k_pass1_vare + pass 2) -> E"}
    # C5's whole build (cb = 16) on the same resident keys, as c4_exact_passes
    import numpy as np
    index = np.empty(n, np.uint64)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    E, vals, sb, used = ctx.mph_build_index_passes(blob, 0, n, 16, 0, offsets=off, addr_base=0x2000, addr_stride=64,
                                                   index=index)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    okb = int(E[-1].item()) & ((1 << 56) - 1) == n
    del E, vals, sb, index, blob, off
    torch.cuda.empty_cache()
    build = {"n_keys": n, "checksum_bits": 16, "passes": used, "keys_per_s": n / dt, "ms": dt * 1e3,
             "check": {"E[m]==n": okb},
             "path": "var-len keys resident in HBM -> bsdb_dev_mph_build_index_passes_var -> GOV structure in "
                     "HBM, index.db slots in host memory"}
    return hist, build


def full_build_cpu(n: int, width: int, threads: int):
    """The same stages on the host cores: oracle hash, bo_gov_build_mt (threads
    over bucket ranges), lookups and the index scatter ("port")."""
    import time as _t
    import numpy as np
    O = _oracle()
    keys = O.gen_keys13_mt(0, n, threads)
    t0 = _t.perf_counter()
    sig = O.hash_fixed_mt(keys, 13, threads)
    t1 = _t.perf_counter()
    rc, E, vals, sb, _ = O.gov_build_mt(sig, width, threads)
    t2 = _t.perf_counter()
    rank = O.lookup_batch_mt(sig, n, E, vals, width, sb, True, threads)
    index = np.zeros(n, ">u8")
    index[rank] = np.arange(n, dtype=np.uint64)
    t3 = _t.perf_counter()
    assert rc == 0
    return {"n_keys": n, "checksum_bits": width, "keys_per_s": n / (t3 - t0), "ms": (t3 - t0) * 1e3,
            "cores": threads, "kind": "port", "cpu_model": O.cpu_model(),
            "stage_ms": {"hash": (t1 - t0) * 1e3, "gov_build_sort_solve_sign": (t2 - t1) * 1e3,
                         "lookup_index_scatter": (t3 - t2) * 1e3}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--num-keys", dest="n", type=int, default=README_N, help="total keys (all ranks)")
    ap.add_argument("--mode", type=int, default=0, help="0 auto/partitioned, 2 direct atomics")
    ap.add_argument("--chunk", type=int, default=0, help="keys per partitioned chunk (0 = default)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may use")
    ap.add_argument("--no-full-build", action="store_true", help="skip the full-build figures")
    ap.add_argument("--e4-devices", type=int, default=1,
                    help="GPUs of the one-process E4 full-build figure (0 = skip it); never more than asked")
    ap.add_argument("--e4-keys", type=int, default=0,
                    help="N>1: keys of the E4 full-build leg over the ranks (0 = C4's per-GPU share x N)")
    ap.add_argument("--e4-reps", type=int, default=1, help="N>1: timed reps of the E4 leg (after one warm rep)")
    ap.add_argument("--e4-timeout", type=float, default=900.0,
                    help="N>1: seconds the E4 leg may take before every rank abandons it (the line is still printed)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend (nccl = RCCL over xGMI; gloo only to rehearse N ranks on one GPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run (one rank per GPU)")
    dev = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    if args.cpu_threads <= 0 and world == 1 and not args.no_cpu:  # (the CPU legs only)
        args.cpu_threads = _oracle().cpu_threads()

    from bsdb_amd import Context
    ctx = Context(dev)
    collective = "rccl-in-abi"
    if world > 1 and args.backend == "nccl":
        # the one collective runs inside the C ABI (bsdb_dev_histogram_finalize,
        # RCCL over xGMI); the 128-byte communicator id travels over the
        # process group once, outside the timed region.  If the library's own
        # communicator cannot be set up on every rank, the same all-reduce
        # runs through torch.distributed (also RCCL), and the line says so.
        # every rank first agrees that it can load RCCL at all: the
        # communicator init below is collective and has no timeout, so a
        # rank that could not join it would leave the others waiting
        avail = torch.tensor([1 if Context.comm_available() else 0], dtype=torch.int32, device="cuda")
        dist.all_reduce(avail, op=dist.ReduceOp.MIN)
        ok_local = 1
        obj = [None]
        if int(avail.item()) == 0:
            pass
        elif rank == 0:
            try:
                obj[0] = Context.comm_unique_id()
            except Exception as e:  # (RCCL not loadable by the library)
                print(f"[bench r0] bsdb_comm_unique_id failed: {e!r}", file=sys.stderr, flush=True)
        if int(avail.item()) != 0:
            dist.broadcast_object_list(obj, src=0)  # every rank joins, id or None
        if obj[0] is None:
            ok_local = 0
        else:
            try:
                ctx.comm_init(world, rank, obj[0])
            except Exception as e:  # recorded in the line, not hidden
                print(f"[bench r{rank}] bsdb_comm_init failed: {e!r}", file=sys.stderr, flush=True)
                ok_local = 0
        flag = torch.tensor([ok_local], dtype=torch.int32, device="cuda")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 0:
            collective = "torch.distributed all_reduce (RCCL)"
    if args.mode:
        ctx.set_histogram_mode(args.mode)
    if args.chunk:
        ctx.set_chunk_keys(args.chunk)

    def log(msg):
        print(f"[bench r{rank}] {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)

    n = args.n
    m = n // 1500 + 1
    lo, hi = shard(n, rank, world)
    nloc = hi - lo
    log(f"allocating {KEY_LEN * nloc / 1e9:.1f} GB of keys ({nloc} keys, m={m})")
    keys = torch.empty(KEY_LEN * nloc + 16, dtype=torch.uint8, device="cuda")
    ctx.gen_keys13(lo, nloc, out=keys)          # synthetic keys written in HBM (untimed)
    torch.cuda.synchronize()
    log("keys generated")
    counts = torch.zeros(m, dtype=torch.int32, device="cuda")
    E = torch.empty(m + 1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def step():
        # local shard histogram, then ONE all-reduce over RCCL/xGMI (N>1)
        if world > 1 and args.backend == "gloo":
            counts.zero_()
            ctx.histogram_fixed(keys, KEY_LEN, m, counts=counts, n=nloc)
            h = counts.cpu()
            dist.all_reduce(h)
            counts.copy_(h)
            ctx.edge_offsets(counts, out=E)
        elif world > 1 and collective != "rccl-in-abi":
            counts.zero_()
            ctx.histogram_fixed(keys, KEY_LEN, m, counts=counts, n=nloc)
            dist.all_reduce(counts)
            ctx.edge_offsets(counts, out=E)
        elif world > 1:
            counts.zero_()
            ctx.histogram_fixed(keys, KEY_LEN, m, counts=counts, n=nloc)
            ctx.histogram_finalize(counts, n, out=E)   # RCCL all-reduce + scan, E[m] == n checked
        else:
            counts.zero_()
            ctx.histogram_fixed(keys, KEY_LEN, m, counts=counts, n=nloc)
            ctx.edge_offsets(counts, out=E)

    for _ in range(args.warmup):
        step()
        torch.cuda.synchronize()
        log("warmup step done")
    ctx.profile_read(ctx.PASS1); ctx.profile_read(ctx.PASS2); ctx.profile_read(ctx.SCAN)
    ctx.set_profiling(True)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ctx.set_profiling(False)
    p1_ms, p1_launches, p1_keys = ctx.profile_read(ctx.PASS1)
    p2_ms, p2_launches, _ = ctx.profile_read(ctx.PASS2)
    sc_ms, _, _ = ctx.profile_read(ctx.SCAN)

    t = torch.tensor([dt, p1_ms, p2_ms], dtype=torch.float64, device="cuda" if args.backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt, p1_ms_max, p2_ms_max = t.tolist()

    # correctness guard on the measured output: every key counted exactly once
    total = int(E[-1].item())
    ok = total == n

    if rank == 0:
        value = n * args.steps / dt
        p1_avg_s = p1_ms / 1e3 / max(p1_launches, 1)
        keys_per_launch = p1_keys / max(p1_launches, 1)
        achieved = KEY_LEN * keys_per_launch / p1_avg_s / 1e9        # GB/s, algorithmic bytes
        # PMC bytes per launch (profiles/pmc_pass1_latest.json), reported only
        # for the library the counters were collected with and the same launch
        # shape; otherwise null (a kernel change re-collects them)
        traffic, traffic_src = None, None
        prof = os.path.join(ROOT, "profiles", "pmc_pass1_latest.json")
        if os.path.exists(prof):
            try:
                pj = json.load(open(prof))
                same_lib = pj.get("library_sha256") == _lib_sha256()
                same_shape = abs(pj.get("keys_per_launch", 0) - keys_per_launch) < 1.0
                traffic_src = {"file": "profiles/pmc_pass1_latest.json", "round": pj.get("round"),
                               "library_sha256": pj.get("library_sha256"), "same_library": same_lib,
                               "same_launch_shape": same_shape}
                if same_lib and same_shape:
                    traffic = pj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        log(f"timed {args.steps} steps: {dt * 1e3 / args.steps:.2f} ms/step")
    full = None
    if rank == 0 and world == 1 and not args.no_full_build:
        # the rest of the build beside the histogram
        # stage: C4's exact index on the resident keys, C5's var-len histogram
        # at full size, the GPU full build at C2 and C1 size, the CPU port at C1
        full = {}
        try:
            full["c4_histogram_single_pass"] = single_pass_ab(ctx, keys, n, m, counts)
        except Exception as e:  # recorded, not faked
            full["c4_histogram_single_pass"] = {"error": repr(e)[:300]}
        log("single-pass A/B done")
        try:
            full["gpu_c4_exact_passes"] = c4_exact_passes(ctx, keys, n, 4)
        except Exception as e:  # recorded, not faked; the headline line is printed regardless
            full["gpu_c4_exact_passes"] = {"error": repr(e)[:300]}
        log("C4 exact full build done")
        del keys
        torch.cuda.empty_cache()
        ctx.release_workspace()
        try:
            full["e2e_c4_host_passes"] = e2e_c4_host_passes(ctx, n, 4)
        except Exception as e:  # recorded, not faked
            full["e2e_c4_host_passes"] = {"error": repr(e)[:300]}
        torch.cuda.empty_cache()
        log("C4 host passes done")
        try:
            full["gpu_c5_varlen_histogram"], full["gpu_c5_full_build_passes"] = c5_varlen_histogram(
                ctx, 4_000_000_000, 5)
        except Exception as e:
            full["gpu_c5_varlen_histogram"] = {"error": repr(e)[:300]}
        log("C5 histogram done")
        full["gpu_c2"] = full_build_gpu(ctx, 100_000_000, 4, 2)
        full["gpu_c1"] = full_build_gpu(ctx, 1_000_000, 4, 3)
        try:
            full["e2e_c2_host_to_disk"] = e2e_host_to_disk(ctx, 100_000_000, 4)
        except OSError as e:  # (no room for 0.8 GB in /tmp: the figure is skipped, not faked)
            full["e2e_c2_host_to_disk"] = {"skipped": str(e)}
        # from the data files: C2 with 8 partitions and with the reference
        # writer's 2 x cores, C3 (approximate index) with 2 x cores
        kv_parts = 2 * usable_cpus()
        for key, kn, parts, approx in (("e2e_c2_kv_to_disk", 100_000_000, 8, False),
                                       ("e2e_c2_kv_to_disk_2xcores", 100_000_000, kv_parts, False),
                                       ("e2e_c3_kv_to_disk", 1_000_000_000, kv_parts, True)):
            try:
                full[key] = e2e_kv_to_disk(ctx, kn, 4, parts, approx)
            except Exception as e:  # recorded, not faked
                full[key] = {"error": repr(e)[:300]}
            log(f"{key} done")
        if args.e4_devices > 0:
            try:
                full["e4_c3_multi_device"] = e4_multi_device(ctx, 1_000_000_000, 4, args.e4_devices)
            except Exception as e:  # recorded, not faked; the headline line is printed regardless
                full["e4_c3_multi_device"] = {"error": repr(e)[:300]}
        if not args.no_cpu:
            full["cpu_c1"] = full_build_cpu(1_000_000, 4, args.cpu_threads)
        log("full-build figures done")
    def make_line(cpu, full):
        return {
            "metric": "index-build keys/s (device-resident), 13B x 13-byte keys; % HBM roofline",
            "value": value,
            "unit": "keys/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (SURVEY.md §8(d) D2 13-byte keys, generated in HBM before timing)",
            "config": {
                "workload": "BASELINE config 4 (README dataset shape, 13-byte keys), histogram stage: "
                            "SpookyHash-short -> bucket -> bucket-occupancy histogram -> edge offsets "
                            "(edgeOffsetAndSeed); the solve/sign/index stages are the full_build figures",
                "n_keys": n, "key_bytes": KEY_LEN, "num_buckets": m,
                "keys_per_gpu": nloc if world == 1 else f"~{n // world}",
                "parallelism": f"key-shard x{world}" + ((" + RCCL all-reduce(histogram)" if args.backend == "nccl"
                                                         else " + gloo all-reduce (rehearsal)") if world > 1 else ""),
                "collective": (collective if args.backend == "nccl" else "gloo") if world > 1 else None,
                "histogram_mode": "atomic" if args.mode == 2 else "partitioned-2pass",
            },
            "roofline": {
                "bound": "hbm", "kernel": "k_pass1 (hash+bucket+partition)",
                "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic, "traffic_source": traffic_src,
                "bytes_per_key": KEY_LEN, "keys_per_launch": keys_per_launch,
                "avg_launch_ms": p1_avg_s * 1e3, "launches": p1_launches,
            },
            "path_roofline_frac": value * KEY_LEN / (HBM_PEAK_GBS * 1e9) / world,
            "kernel_ms_per_step": {"pass1": p1_ms / args.steps, "pass2": p2_ms / args.steps,
                                   "edge_offsets": sc_ms / args.steps},
            "cpu_baseline": cpu,
            "full_build": full,
            "check": {"E[m]==n": ok},
        }

    if world > 1 and not args.no_full_build:
        # the product's full build at N ranks (E4) beside the histogram stage;
        # every rank joins, rank 0 reports (after the headline's keys are freed)
        del keys
        torch.cuda.empty_cache()
        ctx.release_workspace()
        n_e4 = args.e4_keys if args.e4_keys > 0 else -(-README_N * world // 8)
        full = {}
        # A rank that fails inside the leg leaves the others waiting in a
        # collective: a watchdog on every rank abandons the leg after
        # --e4-timeout seconds, rank 0 printing the line (the histogram
        # stage's figures, the leg recorded as timed out) before every rank
        # exits, so a failed leg never costs the headline's line.
        e4_done = threading.Event()
        emitted = threading.Lock()

        def e4_watchdog():
            if e4_done.wait(args.e4_timeout):
                return
            if rank == 0 and emitted.acquire(blocking=False):
                full["e4_ranks_full_build"] = {"error": f"abandoned after {args.e4_timeout:.0f} s: a rank did not finish the leg"}
                print(json.dumps(make_line(None, full)), flush=True)
            os._exit(0)

        threading.Thread(target=e4_watchdog, daemon=True).start()
        try:
            full["e4_ranks_full_build"] = e4_ranks_full_build(ctx, world, rank, args.backend, 4, args.e4_reps, n_e4)
        except Exception as e:  # recorded, not faked; the headline line is printed regardless
            full["e4_ranks_full_build"] = {"error": repr(e)[:300]}
        e4_done.set()
        log("E4 full build over the ranks done")
        if rank == 0 and not emitted.acquire(blocking=False):
            return  # (the watchdog printed the line as the leg ended)
        if rank == 0:
            emitted.release()
    if rank == 0:
        cpu = None
        if not args.no_cpu and world == 1:  # the CPU baseline is an N = 1 figure
            cpu = cpu_baseline(m, args.cpu_seconds, args.cpu_threads)
            log("cpu baseline done")
        print(json.dumps(make_line(cpu, full)), flush=True)
    if "keys" in locals():
        del keys
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        raise SystemExit(f"histogram total {total} != n {n}")


if __name__ == "__main__":
    main()

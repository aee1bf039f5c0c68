// bsdb_capi.hip -- C ABI (include/bsdb_mi355x.h) over the gfx950 kernels.
//
// One context per writer/device: stream, workspace (partition id regions,
// cursors, scan scratch) and host staging, all owned here.  Launch functions
// enqueue only (no hipMalloc/sync on the dev_ path once the workspace has
// grown to the call's size), so a caller can capture them in a hipGraph.
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <sched.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <functional>
#include <chrono>
#include <condition_variable>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <string>
#include <thread>
#include <condition_variable>
#include <deque>
#include <vector>

#include "../../include/bsdb_mi355x.h"
#include "hash_kernels.hip"
#include "fused_kernels.hip"
#include "mph_kernels.hip"
#include "gov_kernels.hip"

using namespace bsdb;

// One slot of the double-buffered host feed: device buffers of a batch and
// the events of its copy and of the compute that read it.
struct FeedSlot {
    void *buf[8] = {};
    size_t cap[8] = {};
    hipEvent_t copied = nullptr, done = nullptr;
    bool used = false;
    std::vector<uint64_t> reb;  // rebased var-len offsets of the batch (host)
};

struct bsdb_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int hist_mode = 0;
    int frontend = 0;  // 13-byte keys: 0 auto (pipelined), 1 LDS-staged, 2 direct per-tile
    int num_cus = 256;
    int d13_variant = 0;  // profiling only (BSDB_D13_VARIANT): results are NOT valid when != 0
    int d13_threads = 512;  // workgroup size of the pipelined 13-byte kernel (BSDB_D13_THREADS=256|512)
    int d13_copies = 8;     // region copies of the binned 13-byte kernel (BSDB_D13_COPIES=8|16|32)
    uint64_t chunk_keys = 0;
    int fused = -1;  // 13-byte keys, single-pass kernel: -1 = what mode 0 picks (BSDB_FUSED), 0 off, 1 on
    int pipe = -1;   // pass 2 of a chunk beside pass 1 of the next: -1 default, 0 off, 1 on (BSDB_PIPE)
    uint64_t pipe_chunks = 0;  // chunks of the pipelined histogram (0 = default; BSDB_PIPE_CHUNKS)
    uint32_t pipe_cus = 0;     // CUs pass 2 keeps while pass 1 runs (0 = default; BSDB_PIPE_P2CUS)
    hipStream_t p2_stream = nullptr;
    hipEvent_t pipe_ev[6] = {};  // [b] pass 1 into buffer b done, [2 + b] buffer b read, [4] start, [5] end
    void *fu_ring = nullptr;  // its ring (FU_SLOTS x 10.5 MB) + sync words
    size_t fu_ring_bytes = 0;
    uint64_t fu_launches = 0;  // single-pass launches enqueued (bsdb_fused_status)
    std::mutex mu;
    // workspace
    void *ids = nullptr;
    size_t ids_bytes = 0;
    uint32_t *cursor = nullptr;   // region fills [nregions][P]
    size_t cursor_bytes = 0;
    uint64_t *p2_pref = nullptr;  // pass-2 plan: prefix of the segment fills
    size_t p2_pref_bytes = 0;
    uint32_t *overflow = nullptr; // 1 word
    uint64_t *scan_part = nullptr;
    size_t scan_part_n = 0;
    // host-API staging: two feed slots (double-buffered uploads on copy_stream)
    FeedSlot feed[2];
    hipStream_t copy_stream = nullptr;
    void *d_out = nullptr;
    size_t d_out_bytes = 0;
    // GOV build workspace
    void *g_sorted = nullptr, *g_counts = nullptr, *g_cursor = nullptr, *g_scratch = nullptr, *g_status = nullptr;
    size_t g_sorted_bytes = 0, g_counts_bytes = 0, g_cursor_bytes = 0, g_scratch_bytes = 0, g_status_bytes = 0;
    void *g_big = nullptr, *g_slabs = nullptr;  // oversized buckets: list, sort + solver slabs
    size_t g_big_bytes = 0, g_slabs_bytes = 0;
    void *g_pay = nullptr;  // F2: input position of each sorted signature
    size_t g_pay_bytes = 0;
    void *g_led = nullptr;  // the solver's seed ledger (SeedLedger)
    size_t g_led_bytes = 0;
    void *g_mid = nullptr;  // mid-size ranges: per-workgroup counts (u16) and bases (u32)
    size_t g_mid_bytes = 0;
    void *g_midscr = nullptr;  // k_gov_solve_mid: dense scratch per workgroup
    size_t g_midscr_bytes = 0;
    // the oversized buckets' solver runs on its own stream beside k_gov_solve
    hipStream_t big_stream = nullptr;
    hipEvent_t big_ev[2] = {nullptr, nullptr};  // [0] inputs ready on s, [1] big solve done
    bool verify = false;
    // ordering of workspace use across streams: the last call's
    // completion event and stream
    hipEvent_t last_ev = nullptr;
    hipStream_t last_stream = nullptr;
    // RCCL rank (bsdb_comm_init) and the finalize packing buffer
    void *comm = nullptr;
    int nranks = 1, rank = 0;
    // live MPHF objects of this context: bsdb_close releases their device
    // arrays and detaches them, so freeing one afterwards is safe
    std::mutex mph_mu;
    std::vector<bsdb_mph *> mphs;
    void *pack = nullptr;
    size_t pack_bytes = 0;
    // live profiling: event pairs per launch, per kind
    bool profiling = false;
    struct Rec { hipEvent_t a, b; int kind; uint64_t keys; };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    hipEvent_t ev() {
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }
};

// A call that uses the context's workspace on stream s first waits for the
// previous such call when that one ran on another stream, and leaves its own
// completion event behind (launches are asynchronous: without this, two dev
// calls on different streams, or a host call on the private stream beside a
// dev call, would race on the shared buffers).
struct Ordered {
    bsdb_ctx *c;
    hipStream_t s;
    Ordered(bsdb_ctx *c_, hipStream_t s_) : c(c_), s(s_) {
        if (c->last_ev && c->last_stream != s) (void)hipStreamWaitEvent(s, c->last_ev, 0);
    }
    ~Ordered() {
        if (!c->last_ev && hipEventCreateWithFlags(&c->last_ev, hipEventDisableTiming) != hipSuccess) c->last_ev = nullptr;
        if (c->last_ev) (void)hipEventRecord(c->last_ev, s);
        c->last_stream = s;
    }
};

// RAII bracket: records an event before and after the launches in its scope.
struct ProfScope {
    bsdb_ctx *c; hipStream_t s; int kind; uint64_t keys; hipEvent_t a = nullptr;
    ProfScope(bsdb_ctx *c_, hipStream_t s_, int k, uint64_t n) : c(c_), s(s_), kind(k), keys(n) {
        if (c->profiling) { a = c->ev(); (void)hipEventRecord(a, s); }
    }
    ~ProfScope() {
        if (!a) return;
        hipEvent_t b = c->ev();
        (void)hipEventRecord(b, s);
        c->recs.push_back({a, b, kind, keys});
    }
};

static void comm_destroy(bsdb_ctx *c);  // capi_comm.hip

namespace {

constexpr uint64_t DEFAULT_CHUNK_KEYS = 1ULL << 32;  // measured: 2^32 286 G keys/s, 2^33 284, one launch (13.2e9) 266

// BSDB_DEBUG=1: every failing HIP call behind an EIO is reported on stderr
// with its source line (the return code alone does not say which call failed)
int hip_fail(hipError_t e, const char *what, int line) {
    static const bool dbg = getenv("BSDB_DEBUG") != nullptr;
    if (dbg) fprintf(stderr, "[bsdb] line %d: %s -> %d (%s)\n", line, what, (int)e, hipGetErrorString(e));
    return BSDB_EIO;
}
#define HIP_OK(x)                                                   \
    do {                                                            \
        const hipError_t e_ = (x);                                  \
        if (e_ != hipSuccess) return hip_fail(e_, #x, __LINE__);    \
    } while (0)

// Device allocation whose failure is an answer, not an error state: HIP
// records a failed hipMalloc as the thread's last error, which the next
// launch check (hipGetLastError) would then report as a failed kernel launch
// (BSDB_EIO long after the ENOMEM was handled).  Cleared here.
template <class T>
hipError_t dmalloc(T **p, size_t bytes) {
    const hipError_t e = hipMalloc(reinterpret_cast<void **>(p), bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
    }
    return e;
}

// Workspace growth.  hipFree waits for the whole device (every stream), so a
// regrowth in the middle of overlapped work (the bucket-range passes, whose
// slice copies to host memory run beside the next pass) serialises it: large
// buffers get 1/64 of headroom, which covers the pass-to-pass spread of the
// per-pass key counts (well under 0.1 % at C4) and so avoids the regrowth.
int grow(void **p, size_t *have, size_t need) {
    if (*have >= need) return BSDB_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    const size_t roomy = need >= (1u << 20) ? need + need / 64 : need;
    if (roomy != need && dmalloc(p, roomy) == hipSuccess) {
        *have = roomy;
        return BSDB_OK;
    }
    if (dmalloc(p, need) != hipSuccess) return BSDB_ENOMEM;
    *have = need;
    return BSDB_OK;
}

// Pinned 32 MiB pieces, pooled for the life of the process: the index-file
// writer stages its pieces through them (write_files, capi_mph.hip).
constexpr size_t XFER_PIECE = 32ull << 20;

struct PinnedPool {
    std::mutex mu;
    std::vector<void *> free_list;
    void *take() {
        {
            std::lock_guard<std::mutex> g(mu);
            if (!free_list.empty()) {
                void *p = free_list.back();
                free_list.pop_back();
                return p;
            }
        }
        void *p = nullptr;
        if (hipHostMalloc(&p, XFER_PIECE, hipHostMallocDefault) == hipSuccess) return p;
        (void)hipGetLastError();  // (as dmalloc: not a launch failure)
        return nullptr;
    }
    void give(void *p) {
        if (!p) return;
        std::lock_guard<std::mutex> g(mu);
        free_list.push_back(p);
    }
};
PinnedPool &pinned_pool() {
    static PinnedPool *pool = new PinnedPool();  // (never destroyed: no hipHostFree after the runtime's teardown)
    return *pool;
}

// Reserves the file blocks of [off, off + len) (fallocate, mode 0): 0 when
// they are reserved, 1 when the file system cannot reserve blocks ahead
// (EOPNOTSUPP: such a file is written with pwrite, never through a mapping),
// -1 when they cannot be had (ENOSPC, a tmpfs size limit ...).  A store into
// a shared mapping of a hole the file system cannot back raises SIGBUS, which
// would kill the process (a JVM included), so every mapped store goes to a
// reserved range.
int file_reserve(int fd, uint64_t off, uint64_t len) {
    if (fd < 0 || !len) return 0;
    int r;
    do {
        r = fallocate(fd, 0, (off_t)off, (off_t)len);
    } while (r != 0 && errno == EINTR);
    if (r == 0) return 0;
    return errno == EOPNOTSUPP || errno == ENOSYS ? 1 : -1;
}

// Faults a mapped index file's pages in, in file order, on one thread (the
// writers follow in file order: the builder's pass slices, write_files'
// pieces): a tmpfs/page-cache page is allocated on its first touch, and 16
// writer threads faulting the same file concurrently measured 0.84 GB/s
// against ~5 GB/s for one thread walking it.  For a file mapping (fd >= 0)
// each 64 MiB step first reserves its blocks (file_reserve) and `ready`
// advances past it, so a writer stores into [0, ready) without a reservation
// of its own (ensure()); a step that cannot be reserved ends the walk and the
// writers reserve their own pieces (and fail cleanly).  MADV_POPULATE_WRITE
// (Linux 5.14) then prefaults without touching the data, and reports failure
// instead of raising SIGBUS; elsewhere (EINVAL: an older kernel) a read of one
// byte per page of a reserved step allocates the page the same way.  An
// anonymous mapping (fd < 0: the builder's record arrays) needs no
// reservation.
struct Populator {
    std::thread th;
    std::atomic<bool> stop{false};
    std::atomic<uint64_t> ready{0};  // bytes from base whose blocks are reserved
    int fd = -1;
    uint64_t file_off = 0;           // the file offset of base
    double seconds = 0;
    Populator() = default;
    Populator(const Populator &) = delete;
    Populator &operator=(const Populator &) = delete;
    ~Populator() { finish(); }
    void start(uint8_t *base, uint64_t bytes, int file_fd = -1, uint64_t base_off = 0) {
        fd = file_fd;
        file_off = base_off;
        if (!base || !bytes || getenv("BSDB_NO_PREFAULT")) return;
        th = std::thread([this, base, bytes] {
            const auto t0 = std::chrono::steady_clock::now();
            // (16 MiB steps: each holds the address-space lock, which other
            // threads' mmap/munmap and thread creation wait for)
            constexpr uint64_t STEP = 16ull << 20;
            constexpr int MADV_POPULATE_WRITE_ = 23;
            bool madv = true;
            for (uint64_t o = 0; o < bytes && !stop.load(std::memory_order_relaxed); o += STEP) {
                const uint64_t k = std::min(STEP, bytes - o);
                if (fd >= 0) {
                    if (file_reserve(fd, file_off + o, k) != 0) break;
                    ready.store(o + k, std::memory_order_release);
                }
                if (madv) {
                    if (madvise(base + o, k, MADV_POPULATE_WRITE_) == 0) continue;
                    if (errno != EINVAL) break;  // (the kernel reports what a store would have faulted on)
                    madv = false;
                }
                for (uint64_t q = 0; q < k; q += 4096) (void)*(volatile const uint8_t *)(base + o + q);
            }
            seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        });
    }
    // whether [off, off + len) from base may be stored into
    bool ensure(uint64_t off, uint64_t len) {
        if (fd < 0 || off + len <= ready.load(std::memory_order_acquire)) return true;
        return file_reserve(fd, file_off + off, len) == 0;
    }
    void finish() {
        stop.store(true);
        if (th.joinable()) th.join();
    }
};

// A synchronous copy on a stream of the calling thread (the pass slices'
// copier threads, the address upload beside the MPHF build).  The runtime's
// own pageable path: a parallel pinned-bounce copy was measured 2 % slower
// for C4's 17.6 GB slices and 37 % slower for host-key uploads.
int copy_on_own_stream(int dev, void *dst, const void *src, size_t bytes, hipMemcpyKind kind) {
    if (bytes == 0) return BSDB_OK;
    hipStream_t s = nullptr;
    hipError_t e = hipSetDevice(dev);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMemcpyAsync(dst, src, bytes, kind, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (s) (void)hipStreamDestroy(s);
    return e == hipSuccess ? BSDB_OK : hip_fail(e, kind == hipMemcpyHostToDevice ? "H2D copy (own stream)" : "D2H copy (own stream)", __LINE__);
}
// H2D of pageable memory through two pooled pinned pieces on the caller's
// stream (the memcpy of piece i + 1 beside the DMA of piece i).  For copies
// that run on several host threads at once (the builder's concurrent adds):
// the runtime's own pageable path serialised them (8 kv.db partitions' adds
// at ~1 GB/s each, profiles/r5/kv/), each thread's bounce copies on its own.
// At most BOUNCE_SLOTS copies bounce at once (BSDB_BOUNCE_SLOTS, default 16:
// <= 1 GiB of page-locked pieces however many threads add); a copy
// that cannot have its pieces (hipHostMalloc refused) takes the runtime's
// pageable path instead of failing the add.
struct BounceSlots {
    std::mutex mu;
    std::condition_variable cv;
    int free_slots;
    BounceSlots() {
        const char *e = getenv("BSDB_BOUNCE_SLOTS");
        const int v = e ? atoi(e) : 16;
        free_slots = v > 0 ? v : 1;
    }
    void acquire() {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [this] { return free_slots > 0; });
        --free_slots;
    }
    void release() {
        {
            std::lock_guard<std::mutex> g(mu);
            ++free_slots;
        }
        cv.notify_one();
    }
};
static BounceSlots &bounce_slots() {
    static BounceSlots *b = new BounceSlots();
    return *b;
}
int h2d_bounce(hipStream_t s, void *dst, const void *src, size_t bytes) {
    if (bytes == 0) return BSDB_OK;
    bounce_slots().acquire();
    void *pin[2] = {pinned_pool().take(), pinned_pool().take()};
    if (!pin[0] || !pin[1]) {  // no page-locked memory to be had: the runtime's pageable copy
        pinned_pool().give(pin[0]);
        pinned_pool().give(pin[1]);
        bounce_slots().release();
        hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        return e == hipSuccess ? BSDB_OK : hip_fail(e, "H2D copy (pageable fallback)", __LINE__);
    }
    hipEvent_t ev[2] = {nullptr, nullptr};
    int rc = BSDB_OK;
    for (int i = 0; i < 2 && !rc; ++i)
        if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) rc = BSDB_EIO;
    bool pending[2] = {false, false};
    for (size_t o = 0, k = 0; o < bytes && !rc; o += XFER_PIECE, ++k) {
        const int i = (int)(k & 1);
        const size_t len = std::min(XFER_PIECE, bytes - o);
        if (pending[i] && hipEventSynchronize(ev[i]) != hipSuccess) rc = BSDB_EIO;  // the piece's buffer is free again
        if (rc) break;
        memcpy(pin[i], (const uint8_t *)src + o, len);
        if (hipMemcpyAsync((uint8_t *)dst + o, pin[i], len, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipEventRecord(ev[i], s) != hipSuccess)
            rc = BSDB_EIO;
        pending[i] = true;
    }
    if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = BSDB_EIO;
    for (int i = 0; i < 2; ++i) {
        pinned_pool().give(pin[i]);
        if (ev[i]) (void)hipEventDestroy(ev[i]);
    }
    bounce_slots().release();
    return rc;
}

int d2h_pageable(int dev, void *dst, const void *src, size_t bytes) {
    return copy_on_own_stream(dev, dst, src, bytes, hipMemcpyDeviceToHost);
}
int h2d_pageable(int dev, void *dst, const void *src, size_t bytes) {
    return copy_on_own_stream(dev, dst, src, bytes, hipMemcpyHostToDevice);
}

// NULL is the HIP null stream (torch's default stream reports handle 0), not
// the context's private stream, which only the host-buffer entry points use.
hipStream_t pick(bsdb_ctx *, void *stream) { return (hipStream_t)stream; }

int launch_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? BSDB_OK : hip_fail(e, "kernel launch", 0);
}

// CPUs this process may use: its affinity mask, capped by a cgroup v2 CPU
// quota (a container's share of a large host shows the host's CPUs in both
// std::thread::hardware_concurrency() and the affinity mask)
int usable_cpus() {
    static const int n = [] {
        int c = (int)std::max(1u, std::thread::hardware_concurrency());
        cpu_set_t cs;
        if (sched_getaffinity(0, sizeof(cs), &cs) == 0) c = std::max(1, CPU_COUNT(&cs));
        if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[32] = {0};
            unsigned long long per = 0;
            if (fscanf(f, "%31s %llu", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0) {
                const unsigned long long quota = strtoull(q, nullptr, 10);
                if (quota > 0) c = std::min<int>(c, (int)std::max<unsigned long long>(1, (quota + per - 1) / per));
            }
            fclose(f);
        }
        return c;
    }();
    return n;
}

// ---- pass-1 dispatch over (source layout, epilogue) ------------------------
// One-tile-per-workgroup launches: tiles * 512 work-items must stay below 2^32
// (a dispatch packet's grid size is 32-bit), so callers split larger key sets.
constexpr uint64_t MAX_TILES_PER_LAUNCH = (1ULL << 32) / P1_THREADS - 1;

template <int EPI>
void launch_pass1(const P1Args &a0, bool var, uint32_t key_len, uint64_t tiles, hipStream_t s, int frontend) {
    if (tiles > MAX_TILES_PER_LAUNCH) {
        // split into launches of whole tiles (keys, offsets and outputs shifted)
        for (uint64_t t0 = 0; t0 < tiles; t0 += MAX_TILES_PER_LAUNCH) {
            const uint64_t nt = std::min(MAX_TILES_PER_LAUNCH, tiles - t0);
            P1Args a = a0;
            const uint64_t k0 = t0 * P1_TILE;
            a.n = std::min<uint64_t>(a0.n - k0, nt * P1_TILE);
            if (var) {
                a.offsets = a0.offsets + k0;
            } else {
                a.keys = a0.keys + k0 * key_len;
                a.blob_bytes = a0.blob_bytes - k0 * key_len;
            }
            if (a.sig) a.sig = a0.sig + 2 * k0;
            launch_pass1<EPI>(a, var, key_len, nt, s, frontend);
        }
        return;
    }
    const P1Args &a = a0;
    const dim3 g((uint32_t)tiles), b(P1_THREADS);
    if (var && frontend == 2) {
        k_pass1<SRC_VAR, EPI, 1, 0><<<g, b, 0, s>>>(a);
    } else if (var) {
        k_pass1<SRC_VARSTAGED, EPI, 1, 0><<<g, b, 0, s>>>(a);
    } else if (key_len == 13 && frontend != 1) {
        k_pass1<SRC_DIRECT13, EPI, 4, 13><<<g, b, 0, s>>>(a);
    } else if (key_len == 13) {
        k_pass1<SRC_STAGED13, EPI, 4, 13><<<g, b, 0, s>>>(a);
    } else if (key_len >= 1 && key_len <= 13) {
        k_pass1<SRC_STAGED, EPI, 4, 0><<<g, b, 0, s>>>(a);
    } else if (key_len >= 14 && key_len <= 26) {
        k_pass1<SRC_STAGED, EPI, 2, 0><<<g, b, 0, s>>>(a);
    } else if (key_len >= 27 && key_len <= 52) {
        k_pass1<SRC_STAGED, EPI, 1, 0><<<g, b, 0, s>>>(a);
    } else {
        k_pass1<SRC_FIXED_DIRECT, EPI, 1, 0><<<g, b, 0, s>>>(a);
    }
}

struct PartPlan {
    uint32_t nparts;     // region bins: bucket >> bin_shift
    uint32_t bin_shift;  // <= PART_SHIFT; bins nest in the 32768-bucket pass-2 partitions
    uint32_t capb;       // k_pass1_d13e: ids per LDS bin
    uint32_t nmain;      // region copies shared by the workgroups of one XCD
    uint32_t ntail;      // 13-byte path: NCOPY regions of the bounds-checked tail kernel
    uint32_t grid_d13;   // persistent workgroups of the 13-byte kernel (0 = generic path)
    uint64_t cap;        // ids per (bin, main region), multiple of 64
    uint64_t cap_tail;   // ids per (bin, tail region), multiple of 64
    size_t ids_elems() const { return (size_t)nparts * (nmain * cap + ntail * cap_tail); }
};

uint64_t round64(double x) { return ((uint64_t)x + 63) & ~63ULL; }

using D13Kernel = void (*)(P1Args, uint64_t);

// The persistent pass-1 kernel a context runs.  Variable-length keys:
// k_pass1_vare (BSDB_D13_VARIANT 1, 4: its profiling variants).  13-byte keys (BSDB_D13_VARIANT): 0 k_pass1_d13e
// (production), 1 its hash-and-bins-only profile (results invalid), 2 the
// round-1 sort kernel k_pass1_d13, 4 k_pass1_d13e with phase stamps over
// counts[] (results invalid).
struct D13Sel {
    D13Kernel k;
    int nt;             // workgroup size
    uint64_t tile;      // keys per tile
    uint32_t maxp;      // partitions (bins) supported
    bool binned;        // runs padded to 8 ids, region copies = d13_copies
    uint32_t bin_ids;   // binned: ids per LDS bin buffer
};
// Fixed key lengths the windowed kernel k_pass1_d13e serves (a key's 16-byte
// window from its aligned start); BSDB_NO_FIXED_WINDOW=1 sends 8/12/16 to the
// var-len kernel instead (A/B switch for measurements).
bool windowed_len(uint32_t key_len) {
    return key_len == 13 || ((key_len == 8 || key_len == 12 || key_len == 16) && !getenv("BSDB_NO_FIXED_WINDOW"));
}

D13Sel d13_select(const bsdb_ctx *c, bool var = false, uint32_t key_len = 13, bool seed0 = false) {
    if (!var && key_len != 13 && windowed_len(key_len)) {
        D13Kernel k = key_len == 8    ? (seed0 ? k_pass1_d13e<0, true, 8> : k_pass1_d13e<0, false, 8>)
                      : key_len == 12 ? (seed0 ? k_pass1_d13e<0, true, 12> : k_pass1_d13e<0, false, 12>)
                                      : (seed0 ? k_pass1_d13e<0, true, 16> : k_pass1_d13e<0, false, 16>);
        return {k, D13E_NT, D13E_TILE, D13E_MAXP, true, D13E_BIN_IDS};
    }
    if (!var && key_len != 13)  // every other fixed length: the var-len kernel on k * L offsets
        return {seed0 ? k_pass1_vare<0, true, true> : k_pass1_vare<0, true>, VARE_NT, VARE_TILE, VARE_MAXP, true,
                VARE_BIN_IDS};
    if (var) {
        D13Kernel k = seed0 ? k_pass1_vare<0, false, true> : k_pass1_vare<0, false>;
        if (c->d13_variant == 1) k = k_pass1_vare<1, false>;
        if (c->d13_variant == 4) k = k_pass1_vare<4, false>;
        if (c->d13_variant == 5) k = k_pass1_vare<5, false>;
        if (c->d13_variant == 6) k = k_pass1_vare<6, false>;
        return {k, VARE_NT, VARE_TILE, VARE_MAXP, true, VARE_BIN_IDS};
    }
    switch (c->d13_variant) {
        case 1: return {k_pass1_d13e<1>, D13E_NT, D13E_TILE, D13E_MAXP, true, D13E_BIN_IDS};
        case 4: return {k_pass1_d13e<4>, D13E_NT, D13E_TILE, D13E_MAXP, true, D13E_BIN_IDS};
        case 12: return {k_pass1_d13e<12>, D13E_NT, D13E_TILE, D13E_MAXP, true, D13E_BIN_IDS};
        case 2:
            if (c->d13_threads == 256) return {k_pass1_d13<256>, 256, 256 * P1_KEYS_PER_THREAD, 512, false, 0};
            return {k_pass1_d13<512>, 512, 512 * P1_KEYS_PER_THREAD, 1024, false, 0};
        default:
            return {seed0 ? k_pass1_d13e<0, true> : k_pass1_d13e<0>, D13E_NT, D13E_TILE, D13E_MAXP, true, D13E_BIN_IDS};
    }
}

// Bins of a binned kernel: the smallest bin_shift with ceil(m >> shift) <=
// sel.maxp, so a tile fills each LDS bin to tile/P on average while a bin
// holds bin_ids/P >= 2.25x that (>= 8 sigma).
bool binned_layout(const D13Sel &sel, uint64_t m, uint32_t &shift, uint32_t &nbins, uint32_t &capb) {
    shift = 0;
    while (shift <= (uint32_t)PART_SHIFT && ((m + (1ULL << shift) - 1) >> shift) > (uint64_t)sel.maxp) ++shift;
    if (shift > (uint32_t)PART_SHIFT) return false;
    nbins = (uint32_t)((m + (1ULL << shift) - 1) >> shift);
    capb = std::min<uint32_t>((sel.bin_ids / nbins) & ~7u, (uint32_t)sel.tile + 8);
    return true;
}

// Region capacities: a bin's expected share per region copy plus 8 sigma and
// two tiles of slack (and, for padded runs, 7 pads per tile); a fill beyond
// cap raises the overflow flag and the chunk is recounted with direct
// atomics.  Layout of the id buffer: [nmain][P][cap], then the tail kernel's
// [ntail][P][cap_tail].
PartPlan plan_partitions(const bsdb_ctx *c, uint64_t chunk, uint64_t m, bool d13, const D13Sel &sel) {
    PartPlan p{};
    const bool binned = d13 && sel.binned;
    p.bin_shift = PART_SHIFT;
    p.nparts = (uint32_t)((m + PART_BUCKETS - 1) / PART_BUCKETS);
    if (binned) binned_layout(sel, m, p.bin_shift, p.nparts, p.capb);
    const double frac = std::min(1.0, (double)(1ULL << p.bin_shift) / (double)m);
    p.nmain = binned ? (uint32_t)c->d13_copies : NCOPY;
    const double e = (double)chunk * frac / p.nmain;
    p.cap = round64(e * 1.02 + 8.0 * std::sqrt(e) + 2 * P1_TILE + 64);
    p.ntail = 0;
    p.cap_tail = 0;
    if (d13) {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sel.k, sel.nt, 0) != hipSuccess || per_cu < 1) per_cu = 1;
        per_cu = std::min(per_cu, 2048 / sel.nt);  // at most 32 waves per CU
        const uint64_t tiles = (chunk + sel.tile - 1) / sel.tile;
        p.grid_d13 = (uint32_t)std::min<uint64_t>(tiles, (uint64_t)c->num_cus * per_cu);
        // measurement aid: fewer persistent workgroups (BSDB_D13_GRID, e.g. CUs left for other work)
        if (const char *v = getenv("BSDB_D13_GRID")) p.grid_d13 = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(p.grid_d13, atoll(v)));
        if (binned) {
            const double tiles_per_copy = (double)tiles / p.nmain + 1;
            p.cap = round64(e * 1.02 + 8.0 * std::sqrt(e) + 7.0 * tiles_per_copy + 2 * P1_TILE + 64);
        }
        // the tail (< 2 tiles of the persistent kernel) goes to k_pass1 in
        // blocks of P1_TILE keys, one region each
        p.ntail = NCOPY;
        p.cap_tail = round64(std::max<uint64_t>(P1_TILE, sel.tile) + 64);
    }
    return p;
}

// The single-pass kernel (fused_kernels.hip) over the whole super-tiles of a
// 13-byte key set: *done = the keys it covers (a multiple of 256 * 16384);
// 0 when the set does not qualify.  Enqueue only.
constexpr uint64_t FU_MIN_SUPER = 4;  // super-tiles per workgroup, at least

int fused13_impl(bsdb_ctx *c, const uint8_t *keys, uint64_t blob_bytes, uint64_t n, uint64_t seed, uint64_t m,
                 uint32_t *counts, hipStream_t s, uint64_t *done) {
    *done = 0;
    const uint64_t per = (uint64_t)FU_OWNERS * FU_TILE;
    if (c->num_cus != FU_OWNERS || m == 0 || m > (uint64_t)FU_OWNERS * (FU_TCAP - 2)) return BSDB_OK;
    // a key's 16-byte window ends 3 bytes past it: whole super-tiles whose
    // windows stay inside the blob
    if (blob_bytes < 3) return BSDB_OK;
    const uint64_t nsuper = std::min(n / per, (blob_bytes - 3) / 13 / per);
    if (nsuper < FU_MIN_SUPER) return BSDB_OK;
    // the owner tables count in u16: keep the mean bucket count far below 2^16
    // (a wrap is detected and recounted, but costs the whole launch)
    if (n / m > 16384) return BSDB_OK;
    static int per_cu = -1;
    if (per_cu < 0 && hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_hist13_fused<true>, FU_NT, 0) != hipSuccess)
        per_cu = 0;
    if (per_cu < 1) return BSDB_OK;  // every workgroup must be resident
    const size_t sync_bytes = FU_SYNC_U64 * sizeof(uint64_t);
    const size_t ring_bytes = (size_t)FU_SLOTS * FU_SLOT_BYTES;
    int variant = 0;
    if (const char *v = getenv("BSDB_FU_VARIANT")) variant = atoi(v);
    int rc = grow(&c->fu_ring, &c->fu_ring_bytes, ring_bytes + sync_bytes);
    if (rc) return rc;
    FusedArgs fa{};
    fa.keys = keys;
    fa.nsuper = nsuper;
    fa.seed = seed;
    fa.mult = (uint32_t)(2 * m);
    fa.m = (uint32_t)m;
    fa.ring = (uint8_t *)c->fu_ring;
    fa.sync = (uint64_t *)((uint8_t *)c->fu_ring + ring_bytes);
    fa.overflow = c->overflow;
    fa.counts = counts;
    HIP_OK(hipMemsetAsync(fa.sync, 0, sync_bytes, s));
    HIP_OK(hipMemsetAsync(c->overflow, 0, sizeof(uint32_t), s));
    ++c->fu_launches;
    {
        ProfScope ps(c, s, 0, nsuper * per);
        // BSDB_FU_VARIANT (profiling, fused_kernels.hip): 1, 2, 4 results invalid, 8 phase stamps
        if (variant == 1) k_hist13_fused<true, 1><<<FU_OWNERS, FU_NT, 0, s>>>(fa);
        else if (variant == 2) k_hist13_fused<true, 2><<<FU_OWNERS, FU_NT, 0, s>>>(fa);
        else if (variant == 4) k_hist13_fused<true, 4><<<FU_OWNERS, FU_NT, 0, s>>>(fa);
        else if (variant == 8) k_hist13_fused<true, 8><<<FU_OWNERS, FU_NT, 0, s>>>(fa);
        else if (seed == 0 && !getenv("BSDB_NO_SEED0"))
            k_hist13_fused<true><<<FU_OWNERS, FU_NT, 0, s>>>(fa);
        else
            k_hist13_fused<false><<<FU_OWNERS, FU_NT, 0, s>>>(fa);
    }
    // an overflow anywhere (adversarial sets): nothing was added; recount
    P1Args af{};
    af.keys = keys;
    af.blob_bytes = blob_bytes;
    af.key_len = 13;
    af.n = nsuper * per;
    af.seed = seed;
    af.multiplier = 2 * m;
    af.counts = counts;
    af.overflow = c->overflow;
    k_overflow_fallback<SRC_FIXED_DIRECT, 0><<<1024, P1_THREADS, 0, s>>>(af);
    if ((rc = launch_status())) return rc;
    *done = nsuper * per;
    return BSDB_OK;
}

bool pipe_wanted(const bsdb_ctx *c) { return c->pipe == 1; }

uint32_t pipe_p2_cus(const bsdb_ctx *c) {
    const uint32_t k = c->pipe_cus ? c->pipe_cus : (uint32_t)c->num_cus / 8;  // 4 per XCD
    return std::max<uint32_t>(1, std::min<uint32_t>(k, (uint32_t)c->num_cus / 2));
}

bool fused_wanted(const bsdb_ctx *c) {
    if (c->hist_mode == 3) return true;
    if (c->hist_mode != 0) return false;
    if (c->fused >= 0) return c->fused == 1;
    return false;
}

int histogram_impl(bsdb_ctx *c, const uint8_t *keys, const uint64_t *offsets, uint64_t blob_bytes,
                   uint32_t key_len, uint64_t n, uint64_t seed, uint64_t m, uint32_t *counts,
                   hipStream_t s) {
    if (n == 0) return BSDB_OK;
    const bool var = offsets != nullptr;
    if (!var && key_len == 13 && fused_wanted(c)) {
        uint64_t done = 0;
        const int rc = fused13_impl(c, keys, blob_bytes, n, seed, m, counts, s, &done);
        if (rc) return rc;
        if (done) return histogram_impl(c, keys + done * 13, nullptr, blob_bytes - done * 13, 13, n - done, seed, m,
                                        counts, s);  // the rest (< one super-tile round): two-pass
    }
    P1Args a{};
    a.keys = keys;
    a.offsets = offsets;
    a.blob_bytes = blob_bytes;
    a.key_len = key_len;
    a.seed = seed;
    a.multiplier = 2 * m;
    a.counts = counts;
    const uint32_t nparts = (uint32_t)((m + PART_BUCKETS - 1) / PART_BUCKETS);
    const bool atomic_mode = c->hist_mode == 2 || nparts > (uint32_t)MAX_PARTS;
    // (mode 3 on a set the fused kernel does not take: the two-pass path)
    if (atomic_mode) {
        a.n = n;
        ProfScope ps(c, s, 0, n);
        launch_pass1<EPI_ATOMIC>(a, var, key_len, (n + P1_TILE - 1) / P1_TILE, s, c->frontend);
        return launch_status();
    }
    uint64_t chunk = c->chunk_keys ? c->chunk_keys : DEFAULT_CHUNK_KEYS;
    chunk = std::max<uint64_t>(P1_TILE, chunk / P1_TILE * P1_TILE);
    chunk = std::min<uint64_t>(chunk, (n + P1_TILE - 1) / P1_TILE * P1_TILE);
    // the persistent kernels: 13-byte keys and variable-length keys
    D13Sel sel = d13_select(c, var, key_len, seed == 0 && !getenv("BSDB_NO_SEED0"));  // (A/B switch for measurements)
    uint32_t bsh = 0, nb = 0, cb = 0;
    const bool windowed = !var && windowed_len(key_len);  // k_pass1_d13e (13 B, or 8 / 12 / 16 B)
    const bool fixed_other = !var && !windowed;
    // (fixed keys over 32 B: a 128-key group would overflow the var-len
    // kernel's LDS stage, so they stay on the one-tile-per-workgroup kernels)
    bool d13 = c->frontend == 0 && !(fixed_other && (key_len == 0 || key_len > 32)) &&
               (sel.binned ? binned_layout(sel, m, bsh, nb, cb) : nparts <= sel.maxp);
    if (!d13 && !var && key_len == 13 && c->frontend == 0 && sel.binned) {
        // more bins than the binned kernel holds (m > 288 * 32768): the
        // round-1 persistent sort kernel (up to 1024 partitions)
        sel = D13Sel{k_pass1_d13<512>, 512, 512 * P1_KEYS_PER_THREAD, 1024, false, 0};
        d13 = nparts <= sel.maxp;
    }
    const bool pipe_pl = pipe_wanted(c) && d13 && windowed && sel.binned;
    if (pipe_pl && !c->chunk_keys) {
        // equal chunks of whole tiles: pass 2 of each beside pass 1 of the next
        const uint64_t nch = c->pipe_chunks ? c->pipe_chunks : 8;
        chunk = std::max<uint64_t>(sel.tile, ((n + nch - 1) / nch + sel.tile - 1) / sel.tile * sel.tile);
    }
    PartPlan pp = plan_partitions(c, chunk, m, d13, sel);
    // the id buffers take at most half of the device memory left (workspace
    // included); the 13-byte kernel addresses one region set (P segments)
    // with 32-bit offsets
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
    const size_t budget = (free_b + c->ids_bytes) / 2 / (pipe_pl ? 2 : 1);
    while (chunk > 2 * P1_TILE && (pp.ids_elems() * sizeof(uint16_t) > budget ||
                                   (uint64_t)pp.nparts * pp.cap >= (1ULL << 32))) {
        chunk = std::max<uint64_t>(P1_TILE, chunk / 2 / P1_TILE * P1_TILE);
        pp = plan_partitions(c, chunk, m, d13, sel);
    }
    const uint32_t R = pp.nmain + pp.ntail;
    // Pass 2 of chunk i overlapped with pass 1 of chunk i + 1 (13-byte
    // windowed keys, several chunks): two id buffers; pass 1 on the caller's
    // stream over all CUs but the ones pass 2 keeps (its workgroups hold 128
    // KiB of LDS, pass 1's 146 KiB: one per CU each, so the two launches
    // split the chip); pass 2 on the context's second stream.  The first
    // pass 1 and the last pass 2 get the whole chip.
    const bool pipe = pipe_wanted(c) && d13 && windowed && sel.binned && n > chunk;
    const int nbuf = pipe ? 2 : 1;
    const size_t ids_per_buf = pp.ids_elems(), cur_per_buf = (size_t)pp.nparts * R;
    int rc = grow(&c->ids, &c->ids_bytes, nbuf * ids_per_buf * sizeof(uint16_t));
    if (rc) return rc;
    rc = grow((void **)&c->cursor, &c->cursor_bytes,
              (nbuf * cur_per_buf + P1_SCRATCH_WG + (size_t)P1_SCRATCH_MAXWG * 1024) * sizeof(uint32_t));
    if (rc) return rc;
    rc = grow((void **)&c->p2_pref, &c->p2_pref_bytes, nbuf * (cur_per_buf + 1) * sizeof(uint64_t));
    if (rc) return rc;
    hipStream_t s2 = s;
    if (pipe) {
        if (!c->p2_stream && hipStreamCreateWithFlags(&c->p2_stream, hipStreamNonBlocking) != hipSuccess) return BSDB_EIO;
        for (auto &e : c->pipe_ev)
            if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return BSDB_EIO;
        s2 = c->p2_stream;
        HIP_OK(hipEventRecord(c->pipe_ev[4], s));  // the caller's earlier work
        HIP_OK(hipStreamWaitEvent(s2, c->pipe_ev[4], 0));
    }
    const uint32_t p2_cus = pipe ? pipe_p2_cus(c) : 0;
    a.scratch = c->cursor + nbuf * cur_per_buf;
    a.cap = pp.cap;
    a.nparts = pp.nparts;
    a.nregions = pp.nmain;
    a.region0 = 0;
    a.ncopy = pp.nmain;
    a.bin_shift = pp.bin_shift;
    a.capb = pp.capb;
    P2Layout L0{};
    L0.cap = pp.cap;
    L0.cap_tail = pp.cap_tail;
    L0.nparts = pp.nparts;
    L0.nmain = pp.nmain;
    L0.ntail = pp.ntail;
    L0.bshift = PART_SHIFT - pp.bin_shift;
    L0.num_buckets = m;
    L0.counts = counts;
    uint64_t i = 0;
    for (uint64_t k0 = 0; k0 < n; k0 += chunk, ++i) {
        const uint64_t nk = std::min(chunk, n - k0);
        const bool first = k0 == 0, last = k0 + nk >= n;
        const uint32_t b = pipe ? (uint32_t)(i & 1) : 0;
        // buffer b's ids, cursors, pass-2 plan and overflow flag
        P1Args ac = a;
        ac.ids = (uint16_t *)c->ids + b * ids_per_buf;
        ac.cursor = c->cursor + b * cur_per_buf;
        ac.overflow = c->overflow + 4 * b;
        uint64_t *pref = c->p2_pref + b * (cur_per_buf + 1);
        P2Layout L = L0;
        L.ids = ac.ids;
        L.cursor = ac.cursor;
        L.overflow = ac.overflow;
        ac.n = nk;
        if (var) {
            ac.offsets = offsets + k0;
        } else {
            ac.keys = keys + k0 * key_len;
            // a window past the chunk reads the next chunk's bytes (the blob
            // goes on): only the blob's end limits the persistent kernel
            ac.blob_bytes = pipe ? blob_bytes - k0 * key_len : nk * key_len;
        }
        if (pipe && i >= 2) HIP_OK(hipStreamWaitEvent(s, c->pipe_ev[2 + b], 0));  // pass 2 of chunk i - 2 read buffer b
        HIP_OK(hipMemsetAsync(ac.cursor, 0, sizeof(uint32_t) * cur_per_buf, s));
        HIP_OK(hipMemsetAsync(ac.overflow, 0, sizeof(uint32_t), s));
        {
            ProfScope ps(c, s, 0, nk);
            const uint64_t tiles = (nk + P1_TILE - 1) / P1_TILE;
            if (d13 && (var || fixed_other)) {
                // full tiles to the persistent kernel, the rest (< 1 of its
                // tiles) to the generic kernel, in the tail regions
                const uint64_t nfast = nk / sel.tile;
                if (nfast) {
                    const uint32_t grid = (uint32_t)std::min<uint64_t>(nfast, pp.grid_d13);
                    sel.k<<<grid, sel.nt, 0, s>>>(ac, nfast);
                }
                const uint64_t done = nfast * sel.tile;
                if (done < nk) {
                    P1Args at = ac;
                    at.n = nk - done;
                    at.ids = ac.ids + (size_t)pp.nmain * pp.nparts * pp.cap;
                    at.cursor = ac.cursor + (size_t)pp.nmain * pp.nparts;
                    at.cap = pp.cap_tail;
                    at.nregions = pp.ntail;
                    if (var) {
                        at.offsets = ac.offsets + done;
                        k_pass1<SRC_VAR, EPI_PARTITION, 1, 0><<<(uint32_t)((at.n + P1_TILE - 1) / P1_TILE), P1_THREADS, 0, s>>>(at);
                    } else {
                        at.keys = ac.keys + done * key_len;
                        at.blob_bytes = at.n * key_len;
                        launch_pass1<EPI_PARTITION>(at, false, key_len, (at.n + P1_TILE - 1) / P1_TILE, s, 0);
                    }
                }
            } else if (d13) {
                // full tiles whose 16-byte windows stay inside the readable
                // blob go to the persistent kernel (a key's window ends 16 - L
                // bytes past it at most); the rest (< 2 of its tiles) to the
                // bounds-checked kernel, in the tail regions
                const uint64_t dtile = sel.tile, over = 16 - key_len;
                uint64_t nfast = 0;
                if (ac.blob_bytes >= over) nfast = std::min(nk / dtile, ((ac.blob_bytes - over) / key_len) / dtile);
                if (nfast) {
                    uint32_t grid = (uint32_t)std::min<uint64_t>(nfast, pp.grid_d13);
                    if (pipe && !first) grid = std::max<uint32_t>(1, std::min<uint32_t>(grid, (uint32_t)c->num_cus - p2_cus));
                    sel.k<<<grid, sel.nt, 0, s>>>(ac, nfast);
                }
                const uint64_t done = nfast * dtile;
                if (done < nk) {
                    P1Args at = ac;
                    at.keys = ac.keys + done * key_len;
                    at.n = nk - done;
                    at.blob_bytes = at.n * key_len;
                    at.ids = ac.ids + (size_t)pp.nmain * pp.nparts * pp.cap;
                    at.cursor = ac.cursor + (size_t)pp.nmain * pp.nparts;
                    at.cap = pp.cap_tail;
                    at.nregions = pp.ntail;
                    launch_pass1<EPI_PARTITION>(at, false, key_len, (at.n + P1_TILE - 1) / P1_TILE, s, 0);
                }
            } else {
                launch_pass1<EPI_PARTITION>(ac, var, key_len, tiles, s, c->frontend);
            }
        }
        if (pipe) {
            HIP_OK(hipEventRecord(c->pipe_ev[b], s));  // pass 1 of chunk i done
            HIP_OK(hipStreamWaitEvent(s2, c->pipe_ev[b], 0));
        }
        {
            ProfScope ps(c, s2, 1, nk);
            k_pass2_plan<<<1, SCAN_THREADS, 0, s2>>>(L, pref);
            const uint32_t g2 = pipe && !last ? p2_cus : (uint32_t)c->num_cus;
            k_pass2b<<<g2, P2_THREADS, 0, s2>>>(L, pref);
        }
        if (var) {
            k_overflow_fallback<SRC_VAR, 0><<<1024, P1_THREADS, 0, s2>>>(ac);
        } else {
            k_overflow_fallback<SRC_FIXED_DIRECT, 0><<<1024, P1_THREADS, 0, s2>>>(ac);
        }
        if (pipe) HIP_OK(hipEventRecord(c->pipe_ev[2 + b], s2));  // buffer b free again
        if ((rc = launch_status())) return rc;
    }
    if (pipe) {
        // the caller's stream continues after the last pass 2
        HIP_OK(hipEventRecord(c->pipe_ev[5], s2));
        HIP_OK(hipStreamWaitEvent(s, c->pipe_ev[5], 0));
    }
    return BSDB_OK;
}

int hash_impl(bsdb_ctx *c, const uint8_t *keys, const uint64_t *offsets, uint64_t blob_bytes, uint32_t key_len,
              uint64_t n, uint64_t seed, uint64_t *sig, hipStream_t s) {
    if (n == 0) return BSDB_OK;
    P1Args a{};
    a.keys = keys;
    a.offsets = offsets;
    a.blob_bytes = blob_bytes;
    a.key_len = key_len;
    a.n = n;
    a.seed = seed;
    a.sig = sig;
    launch_pass1<EPI_SIG>(a, offsets != nullptr, key_len, (n + P1_TILE - 1) / P1_TILE, s, c->frontend);
    return launch_status();
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

// BSDBWriter.put keys are 1..255 bytes (Common.java MAX_KEY_SIZE); a fixed
// layout of 0-byte keys is rejected
bool bad_key_len(uint32_t key_len) { return key_len == 0 || key_len > 255; }

}  // namespace

extern "C" {

int bsdb_abi_version(void) { return BSDB_ABI_VERSION; }

const char *bsdb_strerror(int code) {
    switch (code) {
        case BSDB_OK: return "ok";
        case BSDB_EINVAL: return "invalid argument";
        case BSDB_ENOMEM: return "device out of memory";
        case BSDB_EIO: return "HIP runtime error";
        case BSDB_ENODEV: return "no such HIP device";
        case BSDB_EDUP: return "duplicate key signature";
        case BSDB_ESEEDS: return "exhausted local seeds";
        case BSDB_E2BIG: return "bucket too large for the device solver";
        case BSDB_ECOMM: return "RCCL unavailable or collective failed";
        case BSDB_EFILE: return "file open/read/write failed";
        case BSDB_EVERIFY: return "built MPHF failed the bijection check";
        default: return "unknown error";
    }
}

uint64_t bsdb_num_buckets(uint64_t n) { return n / BUCKET_SIZE + 1; }

int bsdb_open(int device, bsdb_ctx **out) {
    if (!out) return BSDB_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return BSDB_ENODEV;
    bsdb_ctx *c = new (std::nothrow) bsdb_ctx();
    if (!c) return BSDB_ENOMEM;
    c->device = device;
    if (const char *v = std::getenv("BSDB_D13_VARIANT")) c->d13_variant = std::atoi(v);
    if (const char *v = std::getenv("BSDB_FUSED")) c->fused = std::atoi(v) ? 1 : 0;
    if (const char *v = std::getenv("BSDB_PIPE")) c->pipe = std::atoi(v) ? 1 : 0;
    if (const char *v = std::getenv("BSDB_PIPE_CHUNKS")) c->pipe_chunks = std::strtoull(v, nullptr, 10);
    if (const char *v = std::getenv("BSDB_PIPE_P2CUS")) c->pipe_cus = (uint32_t)std::atoi(v);
    if (const char *v = std::getenv("BSDB_D13_THREADS")) c->d13_threads = std::atoi(v) == 256 ? 256 : 512;
    if (const char *v = std::getenv("BSDB_D13_COPIES")) {
        const int k = std::atoi(v);
        c->d13_copies = (k == 16 || k == 32 || k == 64) ? k : 8;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        c->num_cus = cus;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return BSDB_EIO;
    }
    // [0] / [4]: overflow flags of id buffers 0 / 1, [2] / [6]: their fallback
    // counts, [3]: single-pass timeouts
    if (dmalloc(&c->overflow, sizeof(uint32_t) * 8) != hipSuccess ||
        hipMemset(c->overflow, 0, sizeof(uint32_t) * 8) != hipSuccess) {
        bsdb_close(c);
        return BSDB_ENOMEM;
    }
    *out = c;
    return BSDB_OK;
}

static void mph_detach_all(bsdb_ctx *c);

// Frees the grown workspace buffers (they grow again on the next call that
// needs them): the histogram id stream, the GOV build's sorted signatures,
// payloads, scratch, ledger and slabs, the host feed's device buffers.
static void release_workspace(bsdb_ctx *c) {
    for (void **p : {&c->ids, &c->d_out, &c->g_sorted, &c->g_pay, &c->g_scratch, &c->g_led, &c->g_mid, &c->g_slabs,
                     &c->g_big, &c->pack, &c->g_midscr}) {
        (void)hipFree(*p);
        *p = nullptr;
    }
    c->ids_bytes = c->d_out_bytes = c->g_sorted_bytes = c->g_pay_bytes = c->g_scratch_bytes = c->g_led_bytes =
        c->g_mid_bytes = c->g_slabs_bytes = c->g_big_bytes = c->pack_bytes = c->g_midscr_bytes = 0;
    for (auto &f : c->feed) {
        if (f.used) (void)hipEventSynchronize(f.done);
        for (int i = 0; i < 8; ++i) {
            (void)hipFree(f.buf[i]);
            f.buf[i] = nullptr;
            f.cap[i] = 0;
        }
        f.used = false;
    }
}

int bsdb_release_workspace(bsdb_ctx *c) {
    if (!c) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipDeviceSynchronize());
    release_workspace(c);
    return BSDB_OK;
}

int bsdb_close(bsdb_ctx *c) {
    if (!c) return BSDB_EINVAL;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    mph_detach_all(c);
    (void)hipFree(c->ids);
    (void)hipFree(c->cursor);
    (void)hipFree(c->p2_pref);
    (void)hipFree(c->fu_ring);
    if (c->p2_stream) (void)hipStreamSynchronize(c->p2_stream);
    for (hipEvent_t e : c->pipe_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->p2_stream) (void)hipStreamDestroy(c->p2_stream);
    (void)hipFree(c->overflow);
    (void)hipFree(c->scan_part);
    if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
    for (auto &f : c->feed) {
        for (void *p : f.buf) (void)hipFree(p);
        if (f.copied) (void)hipEventDestroy(f.copied);
        if (f.done) (void)hipEventDestroy(f.done);
    }
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    if (c->big_stream) (void)hipStreamSynchronize(c->big_stream);
    for (hipEvent_t e : c->big_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->big_stream) (void)hipStreamDestroy(c->big_stream);
    (void)hipFree(c->d_out);
    (void)hipFree(c->g_sorted);
    (void)hipFree(c->g_counts);
    (void)hipFree(c->g_cursor);
    (void)hipFree(c->g_scratch);
    (void)hipFree(c->g_status);
    (void)hipFree(c->g_big);
    (void)hipFree(c->g_pay);
    (void)hipFree(c->g_led);
    (void)hipFree(c->g_mid);
    (void)hipFree(c->g_slabs);
    (void)hipFree(c->g_midscr);
    (void)hipFree(c->pack);
    comm_destroy(c);
    if (c->last_ev) (void)hipEventDestroy(c->last_ev);
    for (auto &r : c->recs) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
    for (auto e : c->pool) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return BSDB_OK;
}

int bsdb_set_histogram_mode(bsdb_ctx *c, int mode) {
    if (!c || mode < 0 || mode > 3) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    c->hist_mode = mode;
    return BSDB_OK;
}

int bsdb_set_frontend(bsdb_ctx *c, int frontend) {
    if (!c || frontend < 0 || frontend > 2) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    c->frontend = frontend;
    return BSDB_OK;
}

int bsdb_fallback_count(bsdb_ctx *c, uint64_t *out) {
    if (!c || !out) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipDeviceSynchronize());
    uint32_t v[8] = {};
    HIP_OK(hipMemcpy(v, c->overflow, sizeof(v), hipMemcpyDeviceToHost));
    *out = (uint64_t)v[2] + v[6];
    return BSDB_OK;
}

int bsdb_set_pipeline(bsdb_ctx *c, int mode, uint64_t chunks, uint32_t p2_cus) {
    if (!c || mode < -1 || mode > 1) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    c->pipe = mode;
    c->pipe_chunks = chunks;
    c->pipe_cus = p2_cus;
    return BSDB_OK;
}

int bsdb_fused_status(bsdb_ctx *c, uint64_t *launches, uint64_t *timeouts) {
    if (!c || !launches || !timeouts) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    HIP_OK(hipDeviceSynchronize());
    uint32_t v = 0;
    HIP_OK(hipMemcpy(&v, c->overflow + 3, sizeof(v), hipMemcpyDeviceToHost));
    *launches = c->fu_launches;
    *timeouts = v;
    return BSDB_OK;
}

int bsdb_set_chunk_keys(bsdb_ctx *c, uint64_t chunk_keys) {
    if (!c) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    c->chunk_keys = chunk_keys;
    return BSDB_OK;
}

int bsdb_dev_hash_fixed(bsdb_ctx *c, const uint8_t *d_keys, uint32_t key_len, uint64_t n, uint64_t seed,
                        uint64_t *d_sig, void *stream) {
    if (!c || bad_key_len(key_len) || (n && (!d_keys || !d_sig)) || !aligned16(d_keys) || !aligned16(d_sig))
        return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    return hash_impl(c, d_keys, nullptr, n * key_len, key_len, n, seed, d_sig, pick(c, stream));
}

int bsdb_dev_hash_var(bsdb_ctx *c, const uint8_t *d_blob, uint64_t blob_bytes, const uint64_t *d_off, uint64_t n,
                      uint64_t seed, uint64_t *d_sig, void *stream) {
    if (!c || (n && (!d_blob || !d_off || !d_sig)) || !aligned16(d_sig)) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    return hash_impl(c, d_blob, d_off, blob_bytes, 0, n, seed, d_sig, pick(c, stream));
}

int bsdb_dev_histogram_fixed(bsdb_ctx *c, const uint8_t *d_keys, uint32_t key_len, uint64_t n, uint64_t seed,
                             uint64_t m, uint32_t *d_counts, void *stream) {
    if (!c || bad_key_len(key_len) || m == 0 || m > 0x7FFFFFFFULL || (n && (!d_keys || !d_counts)) || !aligned16(d_keys))
        return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, pick(c, stream));
    return histogram_impl(c, d_keys, nullptr, n * key_len, key_len, n, seed, m, d_counts, pick(c, stream));
}

int bsdb_dev_histogram_var(bsdb_ctx *c, const uint8_t *d_blob, uint64_t blob_bytes, const uint64_t *d_off,
                           uint64_t n, uint64_t seed, uint64_t m, uint32_t *d_counts, void *stream) {
    if (!c || m == 0 || m > 0x7FFFFFFFULL || (n && (!d_blob || !d_off || !d_counts))) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, pick(c, stream));
    return histogram_impl(c, d_blob, d_off, blob_bytes, 0, n, seed, m, d_counts, pick(c, stream));
}

static int edge_offsets_impl(bsdb_ctx *c, const uint32_t *d_counts, uint64_t m, uint64_t *d_E, void *stream);

int bsdb_dev_edge_offsets(bsdb_ctx *c, const uint32_t *d_counts, uint64_t m, uint64_t *d_E, void *stream) {
    if (!c || m == 0 || !d_counts || !d_E) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, pick(c, stream));
    return edge_offsets_impl(c, d_counts, m, d_E, stream);
}

static int edge_offsets_impl(bsdb_ctx *c, const uint32_t *d_counts, uint64_t m, uint64_t *d_E, void *stream) {
    const uint64_t nb = (m + SCAN_BLOCK - 1) / SCAN_BLOCK;
    size_t have = c->scan_part_n * sizeof(uint64_t);
    int rc = grow((void **)&c->scan_part, &have, nb * sizeof(uint64_t));
    if (rc) return rc;
    c->scan_part_n = have / sizeof(uint64_t);
    hipStream_t s = pick(c, stream);
    ProfScope ps(c, s, 2, m);
    k_scan_partial<<<(uint32_t)nb, SCAN_THREADS, 0, s>>>(d_counts, m, c->scan_part);
    k_scan_top<<<1, SCAN_THREADS, 0, s>>>(c->scan_part, nb);
    k_scan_final<<<(uint32_t)nb, SCAN_THREADS, 0, s>>>(d_counts, m, c->scan_part, d_E);
    return launch_status();
}

int bsdb_dev_gen_keys13(bsdb_ctx *c, uint64_t first, uint64_t n, uint8_t *d_keys, void *stream) {
    if (!c || (n && !d_keys) || !aligned16(d_keys)) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    if (n == 0) return BSDB_OK;
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, (uint64_t)c->num_cus * 64);
    k_gen_keys13<<<(uint32_t)blocks, 256, 0, pick(c, stream)>>>(first, n, d_keys);
    return launch_status();
}

int bsdb_dev_gen_keys_var(bsdb_ctx *c, uint64_t first, uint64_t n, uint64_t *d_offsets, uint8_t *d_blob,
                          uint64_t blob_cap, void *stream) {
    if (!c || !d_offsets) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    Ordered ord(c, s);
    if (n == 0) {
        HIP_OK(hipMemsetAsync(d_offsets, 0, 8, s));
        return launch_status();
    }
    int rc = grow(&c->g_counts, &c->g_counts_bytes, n * 4);
    if (rc) return rc;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 255) / 256, (uint64_t)c->num_cus * 64);
    k_gen_var_len<<<blocks, 256, 0, s>>>(first, n, (uint32_t *)c->g_counts);
    if ((rc = edge_offsets_impl(c, (const uint32_t *)c->g_counts, n, d_offsets, s))) return rc;
    if (!d_blob) return launch_status();
    uint64_t total = 0;
    HIP_OK(hipMemcpyAsync(&total, d_offsets + n, 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    if (total > blob_cap) return BSDB_EINVAL;
    k_gen_var_fill<<<blocks, 256, 0, s>>>(first, n, d_offsets, d_blob);
    return launch_status();
}

int bsdb_set_profiling(bsdb_ctx *c, int enable) {
    if (!c) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    c->profiling = enable != 0;
    return BSDB_OK;
}

int bsdb_profile_read(bsdb_ctx *c, int kind, double *total_ms, uint64_t *launches, uint64_t *keys) {
    if (!c || !total_ms || !launches || !keys) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    double t = 0;
    uint64_t nl = 0, nk = 0;
    std::vector<bsdb_ctx::Rec> keep;
    for (auto &r : c->recs) {
        if (r.kind != kind) { keep.push_back(r); continue; }
        HIP_OK(hipEventSynchronize(r.b));
        float ms = 0;
        HIP_OK(hipEventElapsedTime(&ms, r.a, r.b));
        t += ms;
        nl += 1;
        nk += r.keys;
        c->pool.push_back(r.a);
        c->pool.push_back(r.b);
    }
    c->recs.swap(keep);
    *total_ms = t;
    *launches = nl;
    *keys = nk;
    return BSDB_OK;
}

static uint32_t grid_for(const bsdb_ctx *c, uint64_t n) {
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, (uint64_t)c->num_cus * 16));
}

// ---- GOV build on the device (A5, A6, A8, A11) -------------------------------
uint64_t bsdb_values_words(uint64_t n) { return (2 * (1 + ((n * 281) >> 8)) + 63) / 64; }

// SolveArgs::spec from BSDB_GOV_SPEC = "K[,P]": at most K seeds of a bucket in
// flight before a speculating workgroup adds one (0: no limit), P = 1: the
// speculative attempts at a lower wave priority.  Default K = 2: at C1 (667
// buckets on 512 workgroups) the solve takes 5.1 ms against 6.4 ms with no
// limit (every extra seed in flight shares a CU with the attempt that decides
// its bucket); the priority did not help (6.6 ms).
static uint32_t gov_spec_policy() {
    uint32_t spec = 2;
    if (const char *v = getenv("BSDB_GOV_SPEC")) {
        const int k = atoi(v);
        spec = (uint32_t)std::max(0, std::min(k, 255));
        if (const char *c = strchr(v, ','); c && atoi(c + 1)) spec |= 0x100u;
    }
    return spec;
}

static void print_gov_profile(const std::vector<uint64_t> &h, uint32_t solve_grid, uint64_t m) {
    const char *names[GP_N] = {"edges", "peel", "greedy", "bfs", "tarjan", "singletons", "dense", "back",
                               "store", "n_seeds", "n_bfs", "n_bfs_pops", "n_dense_rows", "n_dense_max",
                               "n_core", "n_blocks", "n_rows_in_blocks_over_440", "n_scc_sweeps",
                               "n_small_scc_fallbacks", "fvs_select", "fvs_forms", "fvs_gauss_jordan",
                               "n_fail_degenerate", "n_fail_orient", "n_fail_inconsistent", "failed_attempt_cycles",
                               "bfs_flip", "n_bfs_iters", "n_flip_steps", "n_sel_batches", "n_sel_picks",
                               "sel_pick_cycles", "sel_prep_cycles", "n_singular_solved", "n_null_vectors", "n_speculative_lost",
                               "n_fvs_blocks", "n_form_levels", "n_heavy", "gj_columns", "gj_barrier_wait_cycles",
                               "unused", "tarjan_prep", "tarjan_sweeps", "tarjan_compact",
                               "gj_leader_cycles", "gj_follower_cycles", "gj_slot_columns", "gj_leader_columns",
                               "gj_trailing_cycles", "gj_panels"};
    std::vector<double> tot(GP_N, 0.0);
    for (uint32_t w = 0; w < solve_grid; ++w)
        for (int k = 0; k < GP_N; ++k) {
            const double v = (double)h[(size_t)w * GP_N + k];
            tot[k] = k == GP_N_DENSE_MAX ? std::max(tot[k], v) : tot[k] + v;
        }
    fprintf(stderr, "[gov-profile] m=%llu grid=%u", (unsigned long long)m, solve_grid);
    for (int k = 0; k < GP_N; ++k)
        fprintf(stderr, " %s=%.4g", names[k], k == GP_N_DENSE_MAX ? tot[k] : tot[k] / ((k < GP_N_SEEDS || (k >= GP_FVS_SEL && k <= GP_FVS_GJ) || k == GP_FAILED_CYCLES || k == GP_BFS_FLIP || k == GP_SEL_PICK_CYCLES || k == GP_SEL_PREP_CYCLES || (k >= GP_TJ_PREP && k <= GP_TJ_COMPACT)) ? solve_grid : 1));
    fprintf(stderr, "  (cycles: mean per workgroup; counts: totals)\n");
}

struct DevFree {
    void operator()(void *p) const { if (p) (void)hipFree(p); }
};

// Where a GOV build takes its keys from: n_local signatures of the range
// (sig != nullptr), or the keys themselves (fixed length or a var-len blob),
// re-hashed and filtered to the range's buckets (the sequential range builds
// of bsdb_dev_mph_build_index_passes: no signature array for the whole set).
struct GovSrc {
    const uint64_t *sig = nullptr;
    uint64_t n = 0;  // signatures, or keys
    const uint8_t *keys = nullptr;
    const uint64_t *off = nullptr;
    uint64_t blob_bytes = 0;
    uint32_t key_len = 0;
    // (key sources) every bucket's count over the whole key set, when known:
    // a range build then takes its counts from here instead of re-hashing
    const uint32_t *counts_all = nullptr;
};

// A13 fused into the solve: slot r - idx_lo of index_out gets key p's
// byte-reversed address (addr[p] or addr_base + addr_stride * p).
struct GovIndexOut {
    uint64_t *index = nullptr;
    uint64_t idx_lo = 0;
    const uint64_t *addr = nullptr;
    uint64_t addr_base = 0, addr_stride = 0;
    // (optional) called once the range's key count is known, returns the
    // slots' buffer (at least that many), nullptr when it cannot
    std::function<uint64_t *(uint64_t n_local)> slots;
};

extern "C++" {
template <int MODE>
static void launch_sel(bsdb_ctx *c, const GovSrc &src, SelArgs &a, hipStream_t s) {
    const uint32_t grid = grid_for(c, src.n);
    if (!src.off && src.key_len == 13) k_sel<MODE, 0><<<grid, 256, 0, s>>>(a);
    else if (!src.off) k_sel<MODE, 1><<<grid, 256, 0, s>>>(a);
    else k_sel<MODE, 2><<<grid, 256, 0, s>>>(a);
}
}

// A5 + A6 + A8 + A11 over the buckets [b_lo, b_hi) of a GOV structure on
// n_global keys; d_sig = the n_local signatures of that range.  full: a whole
// build (zeroes the outputs first); otherwise the caller zeroed full-size
// outputs and E[b_hi] is cleared again unless b_hi == m (the next range owns it).
// d_rank (optional, F2): the rank of input signature i at d_rank[i], from the
// solve itself.  With a key source the range's keys are found by re-hashing
// every key, and *n_found (optional) returns how many there were.
static int gov_build_impl(bsdb_ctx *c, const GovSrc &src, uint64_t n_global, uint64_t b_lo, uint64_t b_hi,
                          uint64_t e_lo, uint32_t width, uint64_t *d_E, uint64_t *d_values, uint64_t *d_sigbits,
                          int64_t *d_rank, const GovIndexOut &ixo_in, hipStream_t s, bool full, uint64_t *n_found = nullptr) {
    const uint64_t m = n_global / BUCKET_SIZE + 1, nb = b_hi - b_lo;
    const uint32_t mult = (uint32_t)(2 * m);
    const bool from_keys = src.sig == nullptr;
    int rc;
    if ((rc = grow(&c->g_counts, &c->g_counts_bytes, (nb + 1) * 4))) return rc;  // (+1: k_bucket_count_mid's flag)
    if ((rc = grow(&c->g_cursor, &c->g_cursor_bytes, std::max<uint64_t>(nb, 1) * 8))) return rc;
    if ((rc = grow(&c->g_status, &c->g_status_bytes, 16))) return rc;
    uint32_t *counts = (uint32_t *)c->g_counts, *status = (uint32_t *)c->g_status;
    HIP_OK(hipMemsetAsync(counts, 0, (nb + 1) * 4, s));
    HIP_OK(hipMemsetAsync(status, 0, 16, s));
    if (full) HIP_OK(hipMemsetAsync(d_values, 0, bsdb_values_words(n_global) * 8, s));
    uint64_t *Eb = d_E + b_lo;
    SelArgs sel{src.keys, src.off, src.blob_bytes, src.n, src.key_len, mult, (uint32_t)b_lo, (uint32_t)nb,
                counts, nullptr, nullptr, nullptr};
    // mid-size ranges from signatures: per-workgroup counts and bases, no
    // per-key global atomics (k_bucket_count_mid)
    const bool mid = !from_keys && src.n && nb > SMALL_NB && nb <= MID_NB && src.n < (1ULL << 32);
    const uint32_t mid_g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)c->num_cus, src.n / 65536));
    uint16_t *mid_cw = nullptr;
    uint32_t *mid_base = nullptr;
    if (mid) {
        const size_t cw_bytes = ((size_t)mid_g * nb * 2 + 255) & ~(size_t)255;
        if ((rc = grow(&c->g_mid, &c->g_mid_bytes, cw_bytes + (size_t)mid_g * nb * 4))) return rc;
        mid_cw = (uint16_t *)c->g_mid;
        mid_base = (uint32_t *)((uint8_t *)c->g_mid + cw_bytes);
    }
    if (from_keys) {
        if (src.counts_all)
            HIP_OK(hipMemcpyAsync(counts, src.counts_all + b_lo, nb * 4, hipMemcpyDeviceToDevice, s));
        else if (src.n)
            launch_sel<0>(c, src, sel, s);
    } else if (src.n && nb <= SMALL_NB) {
        k_bucket_count_small<<<(uint32_t)((src.n + SMALL_CHUNK - 1) / SMALL_CHUNK), 256, 0, s>>>(src.sig, src.n, mult, (uint32_t)b_lo,
                                                                                               (uint32_t)nb, counts);
    } else if (mid) {
        k_bucket_count_mid<<<mid_g, MID_THREADS, 0, s>>>(src.sig, src.n, mult, (uint32_t)b_lo, (uint32_t)nb, mid_cw,
                                                         counts + nb);
        k_mid_colsum<<<(uint32_t)((nb + 255) / 256), 256, 0, s>>>(mid_cw, mid_g, (uint32_t)nb, counts);
        k_bucket_count_redo<<<1, 256, 0, s>>>(src.sig, src.n, mult, (uint32_t)b_lo, (uint32_t)nb, counts, counts + nb);
    } else if (src.n) {
        k_bucket_count<<<grid_for(c, src.n), 256, 0, s>>>(src.sig, src.n, mult, (uint32_t)b_lo, counts);
    }
    if ((rc = edge_offsets_impl(c, counts, nb, Eb, s))) return rc;  // A6: Eb[0..nb]
    if (e_lo) k_add_base<<<grid_for(c, nb + 1), 256, 0, s>>>(Eb, nb + 1, e_lo);
    uint64_t n_local = src.n;
    if (from_keys) {  // the range's key count: its last offset
        uint64_t eh = 0;
        HIP_OK(hipMemcpyAsync(&eh, Eb + nb, 8, hipMemcpyDeviceToHost, s));
        HIP_OK(hipStreamSynchronize(s));
        n_local = (eh & OFFSET_MASK) - e_lo;
    }
    if (n_found) *n_found = n_local;
    if (e_lo + n_local > n_global) return BSDB_EINVAL;
    GovIndexOut ixo = ixo_in;
    if (ixo.slots && !(ixo.index = ixo.slots(n_local))) return BSDB_ENOMEM;
    if ((rc = grow(&c->g_sorted, &c->g_sorted_bytes, std::max<uint64_t>(n_local, 1) * 16))) return rc;
    uint64_t *pay = nullptr;
    if (d_rank || ixo.index || from_keys) {  // (a key source always records positions)
        if ((rc = grow(&c->g_pay, &c->g_pay_bytes, std::max<uint64_t>(n_local, 1) * 8))) return rc;
        pay = (uint64_t *)c->g_pay;
    }
    const uint32_t big_cap = (uint32_t)(n_local / (GS_CMAX + 1) + 1);
    if ((rc = grow(&c->g_big, &c->g_big_bytes, (size_t)big_cap * 4))) return rc;
    // BSDB_GOV_ONE_PER_CU=1 / BSDB_GOV_PER_CU=k (measurement only): k < GS_PER_CU
    // solver workgroups per CU (grid and LDS padding), to price the others
    int per_cu = GS_PER_CU;
    if (getenv("BSDB_GOV_ONE_PER_CU")) per_cu = 1;
    if (getenv("BSDB_GOV_PER_CU")) per_cu = std::max(1, std::min(GS_PER_CU, atoi(getenv("BSDB_GOV_PER_CU"))));
    const size_t lds_pad = per_cu < GS_PER_CU ? (160 * 1024 / (per_cu + 1) + 1024 - sizeof(SolveLds)) & ~(size_t)1023 : 0;
    const uint32_t solve_grid = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>(nb, (uint64_t)c->num_cus * per_cu));
    if ((rc = grow(&c->g_scratch, &c->g_scratch_bytes, (size_t)solve_grid * solve_scratch_words<SolveLds>() * 8)))
        return rc;
    uint64_t *sorted = (uint64_t *)c->g_sorted;
    k_cursor_init<<<grid_for(c, nb), 256, 0, s>>>(Eb, nb, e_lo, (uint64_t *)c->g_cursor);
    if (from_keys) {
        sel.cursor = (unsigned long long *)c->g_cursor;
        sel.sorted = sorted;
        sel.pay = pay;
        if (src.n) launch_sel<1>(c, src, sel, s);
    } else if (mid) {
        k_mid_colscan<<<(uint32_t)((nb + 255) / 256), 256, 0, s>>>(mid_cw, mid_g, (uint32_t)nb, Eb, e_lo, mid_base);
        k_bucket_scatter_mid<<<mid_g, MID_THREADS, 0, s>>>(src.sig, n_local, mult, (uint32_t)b_lo, (uint32_t)nb, mid_base,
                                                           counts + nb, (unsigned long long *)c->g_cursor, sorted, pay);
    } else if (n_local && nb <= SMALL_NB) {
        k_bucket_scatter_small<<<(uint32_t)((n_local + SMALL_CHUNK - 1) / SMALL_CHUNK), 256, 0, s>>>(
            src.sig, n_local, mult, (uint32_t)b_lo, (uint32_t)nb, (unsigned long long *)c->g_cursor, sorted, pay);
    } else if (n_local) {
        k_bucket_scatter<<<grid_for(c, n_local), 256, 0, s>>>(src.sig, n_local, mult, (uint32_t)b_lo,
                                                              (unsigned long long *)c->g_cursor, sorted, pay);
    }
    const uint32_t grid = grid_for(c, n_local);
    k_bucket_sort<<<(uint32_t)std::min<uint64_t>(nb, (uint64_t)c->num_cus * 8), 256, 0, s>>>(sorted, Eb, nb, e_lo,
                                                                                              status, pay);  // A5
    k_big_list<<<grid_for(c, nb), 256, 0, s>>>(Eb, nb, status, (uint32_t *)c->g_big, big_cap);
    if ((rc = launch_status())) return rc;
    uint32_t st[4] = {0, 0, 0, 0};
    HIP_OK(hipMemcpyAsync(st, status, 16, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    if (st[0] & GOV_DUP) return BSDB_EDUP;
    if (st[0] & GOV_TOO_BIG) return BSDB_E2BIG;
    const uint32_t nbig = std::min(st[3], big_cap);
    // oversized buckets: those up to GM_CMAX keys (all of a random set) in
    // LDS, one workgroup per CU (k_gov_solve_mid); larger ones (st[1]) in
    // global slabs (k_gov_solve_big, 8 workgroups)
    const uint32_t nhuge = std::min(st[1], nbig);
    const uint32_t sort_grid = std::min<uint32_t>(nbig, (uint32_t)c->num_cus);
    const uint32_t mid_grid = std::min<uint32_t>(nbig - nhuge, (uint32_t)c->num_cus);
    const uint32_t big_grid = std::min<uint32_t>(nhuge, 8);
    if (nbig) {
        // per-workgroup slabs for the sort, then the global-slab solver's state
        const size_t sort_bytes = (size_t)sort_grid * GB_CMAX * (16 + 8);  // signatures + payloads
        if ((rc = grow(&c->g_slabs, &c->g_slabs_bytes, std::max(sort_bytes, (size_t)big_grid * big_slab_bytes()))))
            return rc;
        if (mid_grid && (rc = grow(&c->g_midscr, &c->g_midscr_bytes, (size_t)mid_grid * solve_scratch_words<SolveMid>() * 8)))
            return rc;
        k_bucket_sort_big<<<sort_grid, GB_THREADS, 0, s>>>(sorted, Eb, e_lo, (const uint32_t *)c->g_big, nbig,
                                                           (ulonglong2 *)c->g_slabs, status, pay);
    }
    // BSDB_GOV_PROFILE=1: per-phase cycle totals of the solver printed to stderr
    const bool gprof = getenv("BSDB_GOV_PROFILE") != nullptr;
    std::unique_ptr<void, DevFree> prof_buf;
    uint64_t *d_prof = nullptr;
    if (gprof) {
        void *p = nullptr;
        HIP_OK(dmalloc(&p, (size_t)solve_grid * GP_N * 8));
        prof_buf.reset(p);
        d_prof = (uint64_t *)p;
        HIP_OK(hipMemsetAsync(d_prof, 0, (size_t)solve_grid * GP_N * 8, s));
    }
    uint32_t fvs_max = FVS_NH_MAX;
    if (const char *v = getenv("BSDB_GOV_FVS_MAX")) fvs_max = (uint32_t)std::max(2, std::min(atoi(v), (int)FVS_NH_MAX));
    if (getenv("BSDB_GOV_PICK_EXACT")) fvs_max |= 0x80000000u;  // (test aid: the exact-rounds FVS picks)
    if (width && full) HIP_OK(hipMemsetAsync(d_sigbits, 0, ((n_global * width + 63) / 64 + 1) * 8, s));
    // the seed ledger: claim, won, done (u32 per bucket), fail (4 u64 per
    // bucket), zeroed; active (u32 per workgroup), all ones
    const size_t led_zero = (size_t)nb * (3 * 4 + 32);
    if ((rc = grow(&c->g_led, &c->g_led_bytes, led_zero + (size_t)solve_grid * 4 + 64))) return rc;
    SeedLedger led;
    {
        uint8_t *q = (uint8_t *)c->g_led;
        led.fail = (unsigned long long *)q;
        led.claim = (uint32_t *)(q + (size_t)nb * 32);
        led.won = led.claim + nb;
        led.done = led.won + nb;
        led.active = led.done + nb;
        HIP_OK(hipMemsetAsync(q, 0, led_zero, s));
        HIP_OK(hipMemsetAsync(led.active, 0xFF, (size_t)solve_grid * 4, s));
    }
    // A8, with A11 (checksum bits at each rank), F2 (ranks) and A13 (index
    // slots) in the solve
    SolveArgs sa{sorted, b_hi, d_E, d_values, (uint64_t *)c->g_scratch, status, d_prof, fvs_max, b_lo, e_lo,
                 d_sigbits, width, pay, d_rank, ixo.index, ixo.idx_lo, ixo.addr, ixo.addr_base, ixo.addr_stride, led,
                 gov_spec_policy()};
    // zeroing status[2] (the bucket queue) above happens before both launches.
    // The oversized buckets (C2: ~3 of 66 667, 2.8 ms of one workgroup each)
    // are solved on a stream of their own, queued first, so their few
    // workgroups run beside k_gov_solve's instead of after them (they touch
    // other buckets; shared value words and checksum words are OR-ed).
    if (nbig) {
        if (!c->big_stream) {
            HIP_OK(hipStreamCreateWithFlags(&c->big_stream, hipStreamNonBlocking));
            for (hipEvent_t &e : c->big_ev) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        HIP_OK(hipEventRecord(c->big_ev[0], s));
        HIP_OK(hipStreamWaitEvent(c->big_stream, c->big_ev[0], 0));
        if (mid_grid)
            k_gov_solve_mid<<<mid_grid, GS_THREADS, 0, c->big_stream>>>(sa, (const uint32_t *)c->g_big, nbig,
                                                                        (uint64_t *)c->g_midscr);
        if (big_grid)
            k_gov_solve_big<<<big_grid, GS_THREADS, 0, c->big_stream>>>(sa, (const uint32_t *)c->g_big, nbig,
                                                                        (uint8_t *)c->g_slabs, big_slab_bytes());
        HIP_OK(hipEventRecord(c->big_ev[1], c->big_stream));
    }
    // (the phase counters are compiled only into k_gov_solve<true>)
    const void *solve_fn = gprof ? (const void *)k_gov_solve<true> : (const void *)k_gov_solve<false>;
    if (lds_pad) HIP_OK(hipFuncSetAttribute(solve_fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_pad));
    if (gprof)
        k_gov_solve<true><<<solve_grid, GS_THREADS, lds_pad, s>>>(sa);  // A8
    else
        k_gov_solve<false><<<solve_grid, GS_THREADS, lds_pad, s>>>(sa);
    if (nbig) HIP_OK(hipStreamWaitEvent(s, c->big_ev[1], 0));
    if (gprof) {
        std::vector<uint64_t> h((size_t)solve_grid * GP_N);
        HIP_OK(hipMemcpyAsync(h.data(), d_prof, h.size() * 8, hipMemcpyDeviceToHost, s));
        HIP_OK(hipStreamSynchronize(s));
        int occ = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_gov_solve<true>, GS_THREADS, lds_pad);
        fprintf(stderr, "[gov-profile] solver workgroups per CU: %d (LDS %zu B each + %zu padding), grid %u\n", occ,
                sizeof(SolveLds), lds_pad, solve_grid);
        print_gov_profile(h, solve_grid, m);
    }
    const MphView v{d_E, d_values, nullptr, n_global, mult, width};
    if (c->verify && n_local) {
        void *p = nullptr;
        HIP_OK(dmalloc(&p, ((n_local + 63) / 64) * 8));
        std::unique_ptr<void, DevFree> bm(p);
        HIP_OK(hipMemsetAsync(p, 0, ((n_local + 63) / 64) * 8, s));
        k_verify_ranks<<<grid, 256, 0, s>>>(v, sorted, n_local, e_lo, (unsigned long long *)p, status);
        HIP_OK(hipStreamSynchronize(s));
    }
    if (b_hi < m) HIP_OK(hipMemsetAsync(d_E + b_hi, 0, 8, s));  // owned by the next range
    if ((rc = launch_status())) return rc;
    HIP_OK(hipMemcpyAsync(st, status, 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    if (st[0] & GOV_DUP) return BSDB_EDUP;
    if (st[0] & GOV_TOO_BIG) return BSDB_E2BIG;
    if (st[0] & GOV_SEEDS) return BSDB_ESEEDS;
    if (st[0] & GOV_VERIFY) return BSDB_EVERIFY;
    return BSDB_OK;
}

// the signature form used by the existing entry points
static int gov_build_impl(bsdb_ctx *c, const uint64_t *d_sig, uint64_t n_local, uint64_t n_global, uint64_t b_lo,
                          uint64_t b_hi, uint64_t e_lo, uint32_t width, uint64_t *d_E, uint64_t *d_values,
                          uint64_t *d_sigbits, int64_t *d_rank, hipStream_t s, bool full) {
    GovSrc src;
    src.sig = d_sig ? d_sig : reinterpret_cast<const uint64_t *>(16);  // (n_local == 0: never read)
    src.n = n_local;
    return gov_build_impl(c, src, n_global, b_lo, b_hi, e_lo, width, d_E, d_values, d_sigbits, d_rank, GovIndexOut{}, s,
                          full);
}

int bsdb_dev_gov_build(bsdb_ctx *c, const uint64_t *d_sig, uint64_t n, uint32_t width, uint64_t *d_E,
                       uint64_t *d_values, uint64_t *d_sigbits, void *stream) {
    const uint64_t m = n / BUCKET_SIZE + 1;
    if (!c || width > 64 || !d_E || !d_values || (n && !d_sig) || (width && !d_sigbits) || !aligned16(d_sig) ||
        m > 0x7FFFFFFFULL)
        return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    Ordered ord(c, s);
    return gov_build_impl(c, d_sig, n, n, 0, m, 0, width, d_E, d_values, d_sigbits, nullptr, s, true);
}

int bsdb_dev_gov_build_ranks(bsdb_ctx *c, const uint64_t *d_sig, uint64_t n, uint32_t width, uint64_t *d_E,
                             uint64_t *d_values, uint64_t *d_sigbits, int64_t *d_rank, void *stream) {
    const uint64_t m = n / BUCKET_SIZE + 1;
    if (!c || width > 64 || !d_E || !d_values || (n && (!d_sig || !d_rank)) || (width && !d_sigbits) ||
        !aligned16(d_sig) || m > 0x7FFFFFFFULL)
        return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    Ordered ord(c, s);
    return gov_build_impl(c, d_sig, n, n, 0, m, 0, width, d_E, d_values, d_sigbits, d_rank, s, true);
}

int bsdb_dev_gov_build_range(bsdb_ctx *c, const uint64_t *d_sig, uint64_t n_local, uint64_t n_global, uint64_t b_lo,
                             uint64_t b_hi, uint64_t e_lo, uint32_t width, uint64_t *d_E, uint64_t *d_values,
                             uint64_t *d_sigbits, int64_t *d_rank, void *stream) {
    const uint64_t m = n_global / BUCKET_SIZE + 1;
    if (!c || width > 64 || !d_E || !d_values || (n_local && !d_sig) || (width && !d_sigbits) || !aligned16(d_sig) ||
        m > 0x7FFFFFFFULL || b_lo >= b_hi || b_hi > m || n_local > n_global || e_lo + n_local > n_global)
        return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    Ordered ord(c, s);
    return gov_build_impl(c, d_sig, n_local, n_global, b_lo, b_hi, e_lo, width, d_E, d_values, d_sigbits, d_rank, s,
                          false);
}

// The value words and checksum words the range [e_lo, e_lo + n_local) of keys
// writes (store_bucket: words [vo >> 5, (vo + nv + 31) >> 5) of its vertices,
// the checksum fields of its ranks).
int bsdb_gov_range_windows(uint64_t n_global, uint32_t width, uint64_t e_lo, uint64_t n_local, uint64_t *out4) {
    if (!out4 || width > 64 || e_lo + n_local > n_global || n_global > (1ULL << 56)) return BSDB_EINVAL;
    auto vo = [](uint64_t x) { return (x * 281) >> 8; };  // vertexOffset (GOV:315-317)
    const uint64_t v_lo = vo(e_lo), v_hi = vo(e_lo + n_local);
    out4[0] = v_lo >> 5;
    out4[1] = ((v_hi + 31) >> 5) - out4[0];
    out4[2] = width ? (e_lo * width) >> 6 : 0;
    out4[3] = width ? ((((e_lo + n_local) * width) + 63) >> 6) - out4[2] : 0;
    return BSDB_OK;
}

int bsdb_dev_gov_build_window(bsdb_ctx *c, const uint64_t *d_sig, uint64_t n_local, uint64_t n_global, uint64_t b_lo,
                              uint64_t b_hi, uint64_t e_lo, uint32_t width, uint64_t *d_E_win, uint64_t *d_values_win,
                              uint64_t values_w0, uint64_t values_words, uint64_t *d_sigbits_win, uint64_t sig_w0,
                              uint64_t sig_words, int64_t *d_rank, void *stream) {
    const uint64_t m = n_global / BUCKET_SIZE + 1;
    uint64_t need[4];
    if (!c || width > 64 || !d_E_win || !d_values_win || (n_local && !d_sig) || (width && !d_sigbits_win) ||
        !aligned16(d_sig) || m > 0x7FFFFFFFULL || b_lo >= b_hi || b_hi > m || n_local > n_global ||
        e_lo + n_local > n_global || bsdb_gov_range_windows(n_global, width, e_lo, n_local, need) != BSDB_OK)
        return BSDB_EINVAL;
    // the windows must hold every word the range writes
    if (values_w0 > need[0] || values_w0 + values_words < need[0] + need[1] ||
        (width && (sig_w0 > need[2] || sig_w0 + sig_words < need[2] + need[3])))
        return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    Ordered ord(c, s);
    // the range build indexes the structure globally: its bases are moved so
    // that every index it forms lands in the windows (no other word is touched)
    auto shift = [](uint64_t *p, uint64_t first) {
        return reinterpret_cast<uint64_t *>(reinterpret_cast<uintptr_t>(p) - (uintptr_t)first * 8);
    };
    return gov_build_impl(c, d_sig, n_local, n_global, b_lo, b_hi, e_lo, width, shift(d_E_win, b_lo),
                          shift(d_values_win, values_w0), width ? shift(d_sigbits_win, sig_w0) : nullptr, d_rank, s,
                          false);
}

int bsdb_dev_partition_owners(bsdb_ctx *c, const uint64_t *d_sig, const uint64_t *d_payload, uint64_t n, uint64_t m,
                              int nranks, uint64_t *d_out, uint64_t *d_payload_out, uint64_t *h_counts, void *stream) {
    if (!c || nranks < 1 || nranks > OWN_MAXR || m == 0 || m > 0x7FFFFFFFULL || !h_counts ||
        (n && (!d_sig || !d_out)) || !aligned16(d_sig) || !aligned16(d_out) || (!d_payload != !d_payload_out))
        return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    Ordered ord(c, s);
    int rc;
    if ((rc = grow(&c->g_cursor, &c->g_cursor_bytes, std::max<size_t>(c->g_cursor_bytes, OWN_MAXR * 8)))) return rc;
    unsigned long long *cur = (unsigned long long *)c->g_cursor;
    HIP_OK(hipMemsetAsync(cur, 0, OWN_MAXR * 8, s));
    if (n) k_owner_count<<<grid_for(c, n), 256, 0, s>>>(d_sig, n, (uint32_t)(2 * m), m, (uint32_t)nranks, cur);
    if ((rc = launch_status())) return rc;
    uint64_t cnt[OWN_MAXR];
    HIP_OK(hipMemcpyAsync(cnt, cur, nranks * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    uint64_t start[OWN_MAXR], acc = 0;
    for (int g2 = 0; g2 < nranks; ++g2) {
        start[g2] = acc;
        acc += cnt[g2];
        h_counts[g2] = cnt[g2];
    }
    HIP_OK(hipMemcpyAsync(cur, start, nranks * 8, hipMemcpyHostToDevice, s));
    if (n)
        k_owner_scatter<<<grid_for(c, n), 256, 0, s>>>(d_sig, d_payload, n, (uint32_t)(2 * m), m, (uint32_t)nranks, cur,
                                                       d_out, d_payload_out);
    if ((rc = launch_status())) return rc;
    HIP_OK(hipStreamSynchronize(s));  // start[] is a stack buffer
    return BSDB_OK;
}

int bsdb_set_verify(bsdb_ctx *c, int enable) {
    if (!c) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    c->verify = enable != 0;
    return BSDB_OK;
}

// ---- MPHF evaluation (A11-A13) ----------------------------------------------

int bsdb_dev_lookup(bsdb_ctx *c, const uint64_t *d_sig, uint64_t nq, uint64_t n, uint64_t m, const uint64_t *d_E,
                    const uint64_t *d_values, uint32_t width, const uint64_t *d_sigbits, int check, int64_t *d_out,
                    void *stream) {
    if (!c || m == 0 || m > 0x7FFFFFFFULL || width > 64 || (nq && (!d_sig || !d_out || !d_E || !d_values)) ||
        (check && width && !d_sigbits) || !aligned16(d_sig))
        return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    if (nq == 0) return BSDB_OK;
    const MphView v{d_E, d_values, d_sigbits, n, (uint32_t)(2 * m), width};
    k_lookup<<<grid_for(c, nq), 256, 0, pick(c, stream)>>>(v, d_sig, nq, check, d_out);
    return launch_status();
}

int bsdb_dev_sign(bsdb_ctx *c, const uint64_t *d_sig, uint64_t n, uint64_t m, const uint64_t *d_E,
                  const uint64_t *d_values, uint32_t width, uint64_t *d_sigbits, void *stream) {
    if (!c || m == 0 || m > 0x7FFFFFFFULL || width == 0 || width > 64 || (n && (!d_sig || !d_E || !d_values || !d_sigbits)) ||
        !aligned16(d_sig))
        return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    if (n == 0) return BSDB_OK;
    const MphView v{d_E, d_values, nullptr, n, (uint32_t)(2 * m), width};
    k_sign<<<grid_for(c, n), 256, 0, pick(c, stream)>>>(v, d_sig, n, d_sigbits);
    return launch_status();
}

int bsdb_dev_index_scatter(bsdb_ctx *c, const int64_t *d_rank, const uint64_t *d_addr, uint64_t count, uint64_t start,
                           uint64_t len, uint64_t *d_index, const uint64_t *d_value8, const uint8_t *d_value_len,
                           uint8_t *d_index_a, void *stream) {
    if (!c || (count && (!d_rank || !d_addr || !d_index)) || (d_index_a && (!d_value8 || !d_value_len))) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    if (count == 0) return BSDB_OK;
    k_index_scatter<<<grid_for(c, count), 256, 0, pick(c, stream)>>>(d_rank, d_addr, count, start, len, d_index, d_value8,
                                                                      d_value_len, d_index_a);
    return launch_status();
}

}  // extern "C" (the definitions below keep the C linkage of their header declarations)

// ---- host-buffer entry points ---------------------------------------------
// Keys in host memory reach the device through two feed slots: batch i is
// copied on the context's copy stream into slot i % 2 while batch i-1's
// kernels run on the compute stream (c->stream); a slot is refilled only after
// the compute that read it finished (F3: copy and compute overlap).

static int feed_init(bsdb_ctx *c) {
    if (c->copy_stream) return BSDB_OK;
    HIP_OK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    for (auto &f : c->feed) {
        HIP_OK(hipEventCreateWithFlags(&f.copied, hipEventDisableTiming));
        HIP_OK(hipEventCreateWithFlags(&f.done, hipEventDisableTiming));
    }
    return BSDB_OK;
}

// Streams records [0, n) in batches [k0, next(k0)): upload(slot, k0, k1)
// issues the batch's copies on the copy stream, compute(slot, k0, k1) its
// kernels on c->stream.
template <class Next, class Upload, class Compute>
static int feed_batches(bsdb_ctx *c, uint64_t n, Next &&next, Upload &&upload, Compute &&compute) {
    int rc = feed_init(c);
    if (rc) return rc;
    int i = 0;
    for (uint64_t k0 = 0; k0 < n; ++i) {
        const uint64_t k1 = next(k0);
        FeedSlot &f = c->feed[i & 1];
        if (f.used) HIP_OK(hipEventSynchronize(f.done));  // also frees the slot's host staging (reb)
        if ((rc = upload(f, k0, k1))) return rc;
        HIP_OK(hipEventRecord(f.copied, c->copy_stream));
        HIP_OK(hipStreamWaitEvent(c->stream, f.copied, 0));
        if ((rc = compute(f, k0, k1))) return rc;
        HIP_OK(hipEventRecord(f.done, c->stream));
        f.used = true;
        k0 = k1;
    }
    return BSDB_OK;
}

static uint64_t fixed_batch(uint32_t key_len, uint64_t bytes) {
    return std::max<uint64_t>(P1_TILE, bytes / key_len / P1_TILE * P1_TILE);
}

// Fixed-length keys of a batch into slot buffer 0 (+16 B of slack).
static int upload_fixed(bsdb_ctx *c, FeedSlot &f, const uint8_t *h_keys, uint32_t key_len, uint64_t k0, uint64_t k1) {
    int rc = grow(&f.buf[0], &f.cap[0], (size_t)(k1 - k0) * key_len + 16);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(f.buf[0], h_keys + k0 * key_len, (k1 - k0) * key_len, hipMemcpyHostToDevice, c->copy_stream));
    return BSDB_OK;
}

// Batches of variable-length keys: [k0, k1) with at most VAR_BATCH_KEYS keys
// and (unless one key alone is larger) VAR_BATCH_BYTES key bytes.
constexpr uint64_t VAR_BATCH_KEYS = 1ULL << 24;
constexpr uint64_t VAR_BATCH_BYTES = 256ULL << 20;
static uint64_t var_batch_end(const uint64_t *off, uint64_t k0, uint64_t n) {
    uint64_t k1 = std::min(n, k0 + VAR_BATCH_KEYS);
    while (k1 - k0 > 1 && off[k1] - off[k0] > VAR_BATCH_BYTES) k1 = k0 + (k1 - k0) / 2;
    return k1;
}

// A var-len batch: key bytes into slot buffer 0, offsets rebased to the
// batch into buffer 1 (host copy f.reb lives until the slot is reused).
static int upload_var(bsdb_ctx *c, FeedSlot &f, const uint8_t *h_blob, const uint64_t *h_off, uint64_t k0,
                      uint64_t k1) {
    const uint64_t nk = k1 - k0;
    if (h_off[k1] < h_off[k0]) return BSDB_EINVAL;
    const uint64_t bytes = h_off[k1] - h_off[k0];
    int rc = grow(&f.buf[0], &f.cap[0], (size_t)bytes + 16);
    if (rc) return rc;
    if ((rc = grow(&f.buf[1], &f.cap[1], (size_t)(nk + 1) * 8))) return rc;
    f.reb.resize(nk + 1);
    for (uint64_t i = 0; i <= nk; ++i) {
        if (h_off[k0 + i] < h_off[k0] || (i && h_off[k0 + i] < h_off[k0 + i - 1])) return BSDB_EINVAL;
        f.reb[i] = h_off[k0 + i] - h_off[k0];
    }
    HIP_OK(hipMemcpyAsync(f.buf[0], h_blob + h_off[k0], bytes, hipMemcpyHostToDevice, c->copy_stream));
    HIP_OK(hipMemcpyAsync(f.buf[1], f.reb.data(), (nk + 1) * 8, hipMemcpyHostToDevice, c->copy_stream));
    return BSDB_OK;
}

// Accumulates the histogram of n host keys into d_counts (device, c->stream).
static int host_histogram_fixed(bsdb_ctx *c, const uint8_t *h_keys, uint32_t key_len, uint64_t n, uint64_t seed,
                                uint64_t m, uint32_t *d_counts) {
    const uint64_t batch = fixed_batch(key_len, 256ULL << 20);
    return feed_batches(
        c, n, [&](uint64_t k0) { return std::min(n, k0 + batch); },
        [&](FeedSlot &f, uint64_t k0, uint64_t k1) { return upload_fixed(c, f, h_keys, key_len, k0, k1); },
        [&](FeedSlot &f, uint64_t k0, uint64_t k1) {
            return histogram_impl(c, (const uint8_t *)f.buf[0], nullptr, (k1 - k0) * key_len, key_len, k1 - k0, seed, m,
                                  d_counts, c->stream);
        });
}

static int host_histogram_var(bsdb_ctx *c, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n, uint64_t seed,
                              uint64_t m, uint32_t *d_counts) {
    return feed_batches(
        c, n, [&](uint64_t k0) { return var_batch_end(h_off, k0, n); },
        [&](FeedSlot &f, uint64_t k0, uint64_t k1) { return upload_var(c, f, h_blob, h_off, k0, k1); },
        [&](FeedSlot &f, uint64_t k0, uint64_t k1) {
            return histogram_impl(c, (const uint8_t *)f.buf[0], (const uint64_t *)f.buf[1], h_off[k1] - h_off[k0], 0,
                                  k1 - k0, seed, m, d_counts, c->stream);
        });
}

// Signatures of n host keys into d_sig (device, 2n u64).
static int host_hash_fixed_dev(bsdb_ctx *c, const uint8_t *h_keys, uint32_t key_len, uint64_t n, uint64_t seed,
                               uint64_t *d_sig) {
    const uint64_t batch = fixed_batch(key_len, 256ULL << 20);
    return feed_batches(
        c, n, [&](uint64_t k0) { return std::min(n, k0 + batch); },
        [&](FeedSlot &f, uint64_t k0, uint64_t k1) { return upload_fixed(c, f, h_keys, key_len, k0, k1); },
        [&](FeedSlot &f, uint64_t k0, uint64_t k1) {
            return hash_impl(c, (const uint8_t *)f.buf[0], nullptr, (k1 - k0) * key_len, key_len, k1 - k0, seed,
                             d_sig + 2 * k0, c->stream);
        });
}

static int host_hash_var_dev(bsdb_ctx *c, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n, uint64_t seed,
                             uint64_t *d_sig) {
    return feed_batches(
        c, n, [&](uint64_t k0) { return var_batch_end(h_off, k0, n); },
        [&](FeedSlot &f, uint64_t k0, uint64_t k1) { return upload_var(c, f, h_blob, h_off, k0, k1); },
        [&](FeedSlot &f, uint64_t k0, uint64_t k1) {
            return hash_impl(c, (const uint8_t *)f.buf[0], (const uint64_t *)f.buf[1], h_off[k1] - h_off[k0], 0,
                             k1 - k0, seed, d_sig + 2 * k0, c->stream);
        });
}

// counts of a host call: the context's d_out, zeroed, then added to h_counts
static int host_counts_finish(bsdb_ctx *c, uint32_t *d_counts, uint64_t m, uint32_t *h_counts) {
    std::vector<uint32_t> tmp(m);
    HIP_OK(hipMemcpyAsync(tmp.data(), d_counts, m * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    for (uint64_t b = 0; b < m; ++b) h_counts[b] += tmp[b];
    return BSDB_OK;
}

int bsdb_histogram_fixed(bsdb_ctx *c, const uint8_t *h_keys, uint32_t key_len, uint64_t n, uint64_t seed,
                         uint64_t m, uint32_t *h_counts) {
    if (!c || bad_key_len(key_len) || m == 0 || m > 0x7FFFFFFFULL || (n && !h_keys) || !h_counts) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    int rc = grow(&c->d_out, &c->d_out_bytes, m * sizeof(uint32_t));
    if (rc) return rc;
    uint32_t *d_counts = (uint32_t *)c->d_out;
    HIP_OK(hipMemsetAsync(d_counts, 0, m * sizeof(uint32_t), c->stream));
    if ((rc = host_histogram_fixed(c, h_keys, key_len, n, seed, m, d_counts))) return rc;
    return host_counts_finish(c, d_counts, m, h_counts);
}

int bsdb_histogram_var(bsdb_ctx *c, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n, uint64_t seed,
                       uint64_t m, uint32_t *h_counts) {
    if (!c || m == 0 || m > 0x7FFFFFFFULL || (n && (!h_blob || !h_off)) || !h_counts) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    int rc = grow(&c->d_out, &c->d_out_bytes, m * sizeof(uint32_t));
    if (rc) return rc;
    uint32_t *d_counts = (uint32_t *)c->d_out;
    HIP_OK(hipMemsetAsync(d_counts, 0, m * sizeof(uint32_t), c->stream));
    if ((rc = host_histogram_var(c, h_blob, h_off, n, seed, m, d_counts))) return rc;
    return host_counts_finish(c, d_counts, m, h_counts);
}

// Signatures to the host: device batches of <= 2^24 keys in d_out.
template <class Hash>
static int host_sig_batches(bsdb_ctx *c, uint64_t n, uint64_t *h_sig, Hash &&hash) {
    constexpr uint64_t B = 1ULL << 24;
    int rc = grow(&c->d_out, &c->d_out_bytes, (size_t)std::min(n, B) * 16 + 16);
    if (rc) return rc;
    for (uint64_t k0 = 0; k0 < n; k0 += B) {
        const uint64_t nk = std::min(B, n - k0);
        if ((rc = hash(k0, nk, (uint64_t *)c->d_out))) return rc;
        HIP_OK(hipMemcpyAsync(h_sig + 2 * k0, c->d_out, nk * 16, hipMemcpyDeviceToHost, c->stream));
        HIP_OK(hipStreamSynchronize(c->stream));
    }
    return BSDB_OK;
}

int bsdb_hash_fixed(bsdb_ctx *c, const uint8_t *h_keys, uint32_t key_len, uint64_t n, uint64_t seed,
                    uint64_t *h_sig) {
    if (!c || bad_key_len(key_len) || (n && (!h_keys || !h_sig))) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    return host_sig_batches(c, n, h_sig, [&](uint64_t k0, uint64_t nk, uint64_t *d) {
        return host_hash_fixed_dev(c, h_keys + k0 * key_len, key_len, nk, seed, d);
    });
}

int bsdb_hash_var(bsdb_ctx *c, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n, uint64_t seed,
                  uint64_t *h_sig) {
    if (!c || (n && (!h_blob || !h_off || !h_sig))) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    return host_sig_batches(c, n, h_sig, [&](uint64_t k0, uint64_t nk, uint64_t *d) {
        return host_hash_var_dev(c, h_blob, h_off + k0, nk, seed, d);
    });
}


#include "capi_comm.hip"
#include "capi_mph.hip"
#include "capi_multi.hip"
#include "capi_passes.hip"
#include "capi_builder.hip"
#include "capi_kv.hip"

// capi_builder.hip -- the whole build of a key set that streams in from host
// memory, kept in ONE device's HBM and built by bucket-range passes straight
// into the index files.  Included by bsdb_capi.hip after capi_passes.hip.
//   W    = src/main/java/tech/bsdb/write/BSDBWriter.java
//   CBHS = src/main/java/it/unimi/dsi/sux4j/io/ConcurrentBucketedHashStore.java
//   GOV  = src/main/java/it/unimi/dsi/sux4j/mph/GOVMinimalPerfectHashFunctionModified.java
//
// The reference's writer takes records one put at a time (W:75-89): the key
// goes into the bucketed hash store (CBHS:360-395, spilled to 256 segment
// files), the record to a kv.db partition; build() then solves the store
// segment by segment (GOV:385-448, CBHS:852-978) and rescans the data files
// once per index pass (W:107-155).  Its memory stays bounded at README size
// (13.19e9 keys).  Here:
//   add    the keys go straight into HBM (171.5 GB at C4 fits one MI355X) in
//          the caller's batches; the record addresses (unless they are a
//          formula of the add order: fixed-size records of one file) and, for
//          index.approximate, the first value bytes stay in host memory;
//   finish the bucket-range passes of capi_passes.hip over the resident keys
//          (each pass re-hashes every key and solves its range; the solve
//          writes every key's index slot), each pass's slots written to
//          index.db / index_a.db at their offset by a copier thread while the
//          next pass solves.  Addresses that fit HBM beside the keys are read
//          there (the solve stores them itself, or a gather kernel turns the
//          solve's input positions into addresses and value bytes); otherwise
//          the slots carry positions and the copier threads gather the
//          addresses from host memory.
// The MPHF is insertion-order independent (seed 0, buckets sorted by
// signature, CBHS:939-955), and every key's slot receives its own record's
// address, so the files do not depend on the order of the adds: they are
// byte-identical to bsdb_mph_build_index_* on the same records.

// growable host array backed by an anonymous mapping (mremap growth: the
// 100 GB address array of a README-size set is never copied to grow it)
template <class T>
struct HostVec {
    T *p = nullptr;
    uint64_t n = 0, cap = 0;
    bool borrowed = false;
    HostVec() = default;
    HostVec(const HostVec &) = delete;
    HostVec &operator=(const HostVec &) = delete;
    ~HostVec() { release(); }
    void release() {
        if (p && !borrowed && cap) munmap(p, cap * sizeof(T));
        p = nullptr;
        n = cap = 0;
        borrowed = false;
    }
    void borrow(const T *q, uint64_t count) {  // the caller's array, valid for the call
        release();
        p = const_cast<T *>(q);
        n = cap = count;
        borrowed = true;
    }
    bool reserve(uint64_t want) {
        if (want <= cap) return true;
        if (borrowed) return false;
        const uint64_t nc = std::max<uint64_t>({want, cap + cap / 2, 1u << 16});
        void *q = p ? mremap(p, cap * sizeof(T), nc * sizeof(T), MREMAP_MAYMOVE)
                    : mmap(nullptr, nc * sizeof(T), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE,
                           -1, 0);
        if (q == MAP_FAILED) return false;
        // 2 MiB pages where the kernel offers them: the populator and the
        // release walk 512x fewer pages (a 1e8-key build's addresses: 800 MB)
        if (!p) (void)madvise(q, nc * sizeof(T), MADV_HUGEPAGE);
        p = (T *)q;
        cap = nc;
        return true;
    }
    bool append(const T *src, uint64_t k) {
        if (!reserve(n + k)) return false;
        if (k) memcpy(p + n, src, k * sizeof(T));
        n += k;
        return true;
    }
};

struct bsdb_builder {
    bsdb_ctx *c = nullptr;
    uint32_t key_len = 0;  // fixed-length builder; 0 = variable-length keys
    bool approx = false;
    bool stride = false;   // addresses = addr_base + addr_stride * (add order)
    uint64_t addr_base = 0, addr_stride = 0;
    uint64_t n = 0, key_bytes = 0;
    uint8_t *d_keys = nullptr;  // key bytes (+16 B of readable slack past the last key)
    size_t keys_cap = 0;
    uint64_t *d_off = nullptr;  // variable-length keys: offsets[n + 1]
    size_t off_cap = 0;         // entries
    uint32_t uni_len = 0;       // variable-length builder: the common key length while every key has it
    bool uniform = true;
    HostVec<uint64_t> addr, value8;
    HostVec<uint8_t> vlen;
    bool borrowed_records = false;  // one-call forms: the caller's record arrays cover every key
    int failed = BSDB_OK;  // an add that failed part-way leaves the builder unusable
    // an add's copy that failed, recorded before the add releases grow_mu (the
    // add takes mu for `failed` only afterwards, when a finish may hold it):
    // finish reads it once it holds grow_mu exclusively
    std::atomic<int> copy_failed{BSDB_OK};
    bool finished = false;
    // Adds may come from several threads (put() threads, the kv.db scan
    // threads).  mu is held only to RESERVE an add's ranges (its keys' index
    // range and key bytes, room in the key area and the record arrays); the
    // copies into those ranges then run outside it, concurrently, each
    // holding grow_mu shared.  A growth of the key area or of the record
    // arrays (which may move them) takes grow_mu exclusively, so it waits for
    // the copies in flight.  Lock order: mu, then grow_mu, then the context's.
    std::mutex mu;
    std::shared_mutex grow_mu;
    // the record arrays' pages, populated in the background from the open
    // (first-touch faults of ~2 µs a page were most of an add's time)
    Populator pop_addr, pop_v8;
    // Spill mode: keys beyond the device's key area.  The
    // reference bounds a README-size build by spilling every key's signature
    // (sig0, sig1, record rank: 24 B, CBHS:379-395) to one of 256 segment
    // files by sig0's top byte and solving segment by segment (CBHS:852-978).
    // When an add does not fit the device key area (dev_key_cap, or an HBM
    // allocation fails), the resident keys are hashed on the device and moved
    // the same way into 256 host segments of (sig0, sig1) + add position, the
    // key area is released, and every later add is hashed on the device and
    // appended there; the finish uploads each pass's segments (section
    // "spill" below).
    bool spill = false;
    uint64_t dev_key_cap = ~0ull;  // key-area bytes (BSDB_BUILDER_DEVICE_KEY_BYTES: a test knob)
    HostVec<ulonglong2> seg_sig[256];
    HostVec<uint64_t> seg_pos[256];
    void *d_stage = nullptr;       // spill adds: the batch's keys, offsets, signatures, segment order
    size_t stage_cap = 0;
    // The records' addresses (and index_a.db value bytes) on the device as
    // well, uploaded by each add beside its keys, when they fit an eighth of
    // the free HBM at the open: the finish then starts without their upload
    // (C2 from kv.db: 0.1 s of 0.42).  Dropped when they cannot grow.
    bool dev_rec = false;
    void *d_raddr = nullptr, *d_rv8 = nullptr, *d_rvl = nullptr;
    size_t raddr_cap = 0, rv8_cap = 0, rvl_cap = 0;
    std::atomic<int> copying{0};   // adds copying right now (> 1: each through pinned pieces)
    std::atomic<uint64_t> add_copy_ns{0}, add_rec_ns{0};  // (BSDB_BUILDER_PROFILE)
    void stop_prefault() {
        pop_addr.finish();
        pop_v8.finish();
    }
    // called by the finish once its files and device arrays are allocated
    // (the kv.db build holds its partitions' release until then)
    std::function<void()> on_opened;
    ~bsdb_builder() { stop_prefault(); }
};

namespace {

// index.approximate slot (W:140-142): the first min(len, 8) value bytes, the
// rest zero -- the same bytes k_index_scatter stores one by one
__device__ __forceinline__ uint64_t value_slot(uint64_t v, uint32_t len) {
    return len >= 8 ? v : v & ((1ULL << (8 * len)) - 1);
}

// The solve stored each key's input position (byte-reversed, the form it
// stores addresses in) at its slot; this turns a pass's slots into the
// byte-reversed record addresses (REVERSE_ORDER, W:138-139) and, for
// index.approximate, the value slots.  Reads are random (one address and
// value per slot), writes coalesced.
__global__ __launch_bounds__(256) void k_slot_gather(uint64_t *slots, uint64_t nl, const uint64_t *addr,
                                                     uint64_t addr_base, uint64_t addr_stride, const uint64_t *value8,
                                                     const uint8_t *vlen, uint64_t *slots_a) {
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nl; i += step) {
        const uint64_t p = __builtin_bswap64(slots[i]);
        slots[i] = __builtin_bswap64(addr ? addr[p] : addr_base + addr_stride * p);
        if (slots_a) slots_a[i] = value_slot(value8[p], vlen[p]);
    }
}

// offsets of fixed-length keys appended to a variable-length builder
__global__ __launch_bounds__(256) void k_fill_offsets(uint64_t *off, uint64_t count, uint64_t base, uint32_t len) {
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += step) off[i] = base + (i + 1) * len;
}

// Device buffer that keeps its first `used` bytes when it grows (a new
// allocation + a device copy; the add batches normally fit the capacity the
// builder was opened with).
int dev_reserve(bsdb_ctx *c, void **p, size_t *cap, size_t used, size_t need, size_t limit = ~(size_t)0) {
    if (need <= *cap) return BSDB_OK;
    void *q = nullptr;
    size_t nc = std::max(need, std::min(limit, *cap + *cap / 2));
    if (dmalloc(&q, nc) != hipSuccess) {
        nc = need;
        if (dmalloc(&q, nc) != hipSuccess) return BSDB_ENOMEM;
    }
    if (used) HIP_OK(hipMemcpyAsync(q, *p, used, hipMemcpyDeviceToDevice, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    (void)hipFree(*p);
    *p = q;
    *cap = nc;
    return BSDB_OK;
}

// Host-side slot transform of the host-gather mode: turns a piece of k
// position slots into address slots in place and (piece_a != nullptr) fills
// the matching index_a.db slots.
using SlotXform = std::function<void(uint64_t *piece, uint64_t k, uint64_t *piece_a)>;

// An index file being written: its descriptor and, for a regular file, a
// shared mapping of it.  Parallel pwrite()s to one file serialise on the
// file's inode lock (a tmpfs or page-cache write holds it for the whole
// copy: 8 threads wrote C4's 105 GB index at ~2.2 GB/s), while stores into
// a shared mapping fault pages in concurrently.
struct OutFile {
    int fd = -1;
    uint8_t *map = nullptr;
    uint64_t bytes = 0;
    Populator *pop = nullptr;  // the mapping's populator: stores go to reserved blocks only (file_reserve)
};

// nl slots of a device buffer to byte 8 * slot0 of f (W:166-179 writes <= 128
// MiB at a time; here 32 MiB pieces handled by up to 16 threads, each with two
// pinned buffers: the D2H of its next piece runs while it stores the current
// one into the mapping, or pwrite()s it when the file is not mapped).  xf
// (optional) transforms each piece on the host first; with fa it also yields
// index_a.db's piece (straight into fa's mapping when there is one).
int write_slots(int device, const OutFile &f, const uint64_t *d_src, uint64_t nl, uint64_t slot0, const SlotXform *xf,
                const OutFile *fa) {
    if (nl == 0) return BSDB_OK;
    constexpr uint64_t PIECE = XFER_PIECE / 8;  // slots
    const int ncpu = usable_cpus();
    const uint64_t npieces = (nl + PIECE - 1) / PIECE;
    const uint64_t T = std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)16, (uint64_t)ncpu, npieces}));
    std::atomic<int> rc{BSDB_OK};
    auto put = [&](const OutFile &o, const void *buf, uint64_t bytes, uint64_t off) {
        if (o.map) {
            if (off + bytes > o.bytes) return false;
            // (an unreserved hole would raise SIGBUS on a full file system)
            if (o.pop ? !o.pop->ensure(off, bytes) : file_reserve(o.fd, off, bytes) != 0) return false;
            memcpy(o.map + off, buf, bytes);
            return true;
        }
        uint64_t w = 0;
        while (w < bytes) {
            const ssize_t r = pwrite(o.fd, (const uint8_t *)buf + w, bytes - w, (off_t)(off + w));
            if (r <= 0) return false;
            w += (uint64_t)r;
        }
        return true;
    };
    auto work = [&](uint64_t t) {
        hipStream_t st = nullptr;
        void *pin[2] = {nullptr, nullptr};
        hipEvent_t done[2] = {nullptr, nullptr};
        std::vector<uint64_t> a_piece;
        bool ok = hipSetDevice(device) == hipSuccess && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
        for (int i = 0; i < 2 && ok; ++i)
            ok = (pin[i] = pinned_pool().take()) != nullptr &&
                 hipEventCreateWithFlags(&done[i], hipEventDisableTiming) == hipSuccess;
        if (ok && xf && fa && !fa->map) {
            try {
                a_piece.resize(PIECE);
            } catch (const std::bad_alloc &) {
                ok = false;
            }
        }
        auto len_of = [&](uint64_t j) { return std::min<uint64_t>(PIECE, nl - j * PIECE); };
        auto issue = [&](uint64_t j, int i) {
            return hipMemcpyAsync(pin[i], d_src + j * PIECE, len_of(j) * 8, hipMemcpyDeviceToHost, st) == hipSuccess &&
                   hipEventRecord(done[i], st) == hipSuccess;
        };
        if (ok && t < npieces) ok = issue(t, 0);
        int k = 0;
        for (uint64_t j = t; ok && j < npieces; j += T, ++k) {
            const int i = k & 1;
            if (j + T < npieces) ok = issue(j + T, i ^ 1);
            ok = ok && hipEventSynchronize(done[i]) == hipSuccess;
            if (!ok) break;
            const uint64_t len = len_of(j), off = 8 * (slot0 + j * PIECE);
            uint64_t *piece = (uint64_t *)pin[i];
            uint64_t *pa = nullptr;
            if (xf && fa) {
                if (fa->map && (off + len * 8 > fa->bytes ||
                                (fa->pop ? !fa->pop->ensure(off, len * 8) : file_reserve(fa->fd, off, len * 8) != 0)))
                    ok = false;
                pa = fa->map ? reinterpret_cast<uint64_t *>(fa->map + off) : a_piece.data();
            }
            if (ok && xf) (*xf)(piece, len, pa);
            if (!ok || !put(f, piece, len * 8, off) || (pa && !fa->map && !put(*fa, pa, len * 8, off))) {
                rc.store(BSDB_EFILE);
                ok = false;
            }
        }
        if (st) ok = hipStreamSynchronize(st) == hipSuccess && ok;
        if (!ok) {
            int expect = BSDB_OK;
            rc.compare_exchange_strong(expect, BSDB_EIO);
        }
        for (int i = 0; i < 2; ++i) {
            pinned_pool().give(pin[i]);
            if (done[i]) (void)hipEventDestroy(done[i]);
        }
        if (st) (void)hipStreamDestroy(st);
    };
    std::vector<std::thread> th;
    for (uint64_t t = 1; t < T; ++t) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
    (void)hipSetDevice(device);
    return rc.load();
}

int builder_check_records(const bsdb_builder *b, uint64_t count, const uint64_t *h_addr, const uint64_t *h_value8,
                          const uint8_t *h_vlen) {
    if (!count || b->borrowed_records) return BSDB_OK;
    if (!b->stride && !h_addr) return BSDB_EINVAL;
    if (b->approx && (!h_value8 || !h_vlen)) return BSDB_EINVAL;
    return BSDB_OK;
}

// The lengths of a batch of variable-length keys: checked non-decreasing,
// and whether they all equal one length (*len, or 0xFFFFFFFF when they
// differ).  No builder state: callers may run it outside the lock.
int var_batch_lengths(const uint64_t *h_off, uint64_t count, uint32_t *len) {
    uint32_t l0 = count ? (uint32_t)std::min<uint64_t>(h_off[1] - h_off[0], 0xFFFFFFFEu) : 0;
    bool same = true;
    for (uint64_t i = 0; i < count; ++i) {
        if (h_off[i + 1] < h_off[i]) return BSDB_EINVAL;
        same = same && h_off[i + 1] - h_off[i] == l0;
    }
    *len = same ? l0 : 0xFFFFFFFFu;
    return BSDB_OK;
}

// offsets of a batch rebased onto the resident blob on the device:
// off[i] = h_off[i+1] - o0 + base, uploaded as they are and shifted here
__global__ __launch_bounds__(256) void k_rebase_offsets(uint64_t *off, uint64_t count, uint64_t shift) {
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += step) off[i] += shift;
}

// One batch of an add: fixed-length keys (keys, key_len) or variable-length
// ones (the blob indexed by off[0..count], lengths checked by
// var_batch_lengths; uni = their common length or 0xFFFFFFFF).
struct AddBatch {
    const uint8_t *keys = nullptr;
    const uint64_t *off = nullptr;
    uint32_t key_len = 0;
    uint32_t uni = 0xFFFFFFFFu;
    uint64_t count = 0;
    uint64_t o0() const { return off ? off[0] : 0; }
    uint64_t bytes() const { return off ? off[count] - off[0] : (uint64_t)key_len * count; }
    const uint8_t *first() const { return keys + o0(); }
};

// ---- spill mode (keys beyond the device's key area) -------------------------
// 256 segments by sig0's top byte, as CBHS:379-395 (sig0 >>> 56); a key's
// entry is its (sig0, sig1) and its add position (its record's rank in the
// add order, CBHS:386-388's "data" word).
constexpr uint32_t NSEG = 256;
constexpr uint64_t SEG_CHUNK = 256 * 16;  // keys a workgroup places per round

__global__ __launch_bounds__(256) void k_seg_count(const ulonglong2 *sig, uint64_t n, uint32_t *counts) {
    __shared__ uint32_t c[NSEG];
    c[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += step) atomicAdd(&c[sig[i].x >> 56], 1u);
    __syncthreads();
    if (c[threadIdx.x]) atomicAdd(counts + threadIdx.x, c[threadIdx.x]);
}

// entries grouped by segment: per round a workgroup ranks its SEG_CHUNK keys
// in LDS and reserves one run per segment (one cursor atomic each); the order
// inside a segment is arbitrary (the solve sorts each bucket, CBHS:939-955)
__global__ __launch_bounds__(256) void k_seg_scatter(const ulonglong2 *sig, uint64_t n, uint64_t pos0,
                                                     unsigned long long *cursor, ulonglong2 *out_sig, uint64_t *out_pos) {
    __shared__ uint32_t c[NSEG];
    __shared__ unsigned long long base[NSEG];
    for (uint64_t lo = (uint64_t)blockIdx.x * SEG_CHUNK; lo < n; lo += (uint64_t)gridDim.x * SEG_CHUNK) {
        c[threadIdx.x] = 0;
        __syncthreads();
        uint32_t seg[16], rank[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint64_t i = lo + (uint64_t)j * 256 + threadIdx.x;
            seg[j] = i < n ? (uint32_t)(sig[i].x >> 56) : 0;
            rank[j] = i < n ? atomicAdd(&c[seg[j]], 1u) : 0;
        }
        __syncthreads();
        if (c[threadIdx.x]) base[threadIdx.x] = atomicAdd(cursor + threadIdx.x, (unsigned long long)c[threadIdx.x]);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint64_t i = lo + (uint64_t)j * 256 + threadIdx.x;
            if (i < n) {
                const uint64_t p = base[seg[j]] + rank[j];
                out_sig[p] = sig[i];
                out_pos[p] = pos0 + i;
            }
        }
        __syncthreads();
    }
}

// the keys of buckets [b_lo, b_hi) among uploaded segment entries (a segment
// at either end of the range also holds keys of the neighbouring buckets)
__global__ __launch_bounds__(256) void k_range_compact(const ulonglong2 *in, const uint64_t *in_pos, uint64_t n,
                                                       uint32_t mult, uint32_t b_lo, uint32_t b_hi, ulonglong2 *out,
                                                       uint64_t *out_pos, unsigned long long *count) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t i0 = (uint64_t)blockIdx.x * 256; i0 < n; i0 += (uint64_t)gridDim.x * 256) {
        const uint64_t i = i0 + threadIdx.x;
        bool keep = false;
        ulonglong2 s{0, 0};
        if (i < n) {
            s = in[i];
            const uint32_t b = bucket_of_w(w64(s.x), mult);
            keep = b >= b_lo && b < b_hi;
        }
        const uint64_t bal = __builtin_amdgcn_ballot_w64(keep);
        if (!bal) continue;
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(count, (unsigned long long)__builtin_popcountll(bal));
        const uint32_t lo32 = (uint32_t)__shfl((int)(uint32_t)base, 0, 64);
        const uint32_t hi32 = (uint32_t)__shfl((int)(uint32_t)(base >> 32), 0, 64);
        if (keep) {
            const uint64_t p = (((uint64_t)hi32 << 32) | lo32) + (uint64_t)__builtin_popcountll(bal & ((1ULL << lane) - 1));
            out[p] = s;
            out_pos[p] = in_pos[i];
        }
    }
}

// Device scratch of the spill path (grown, kept until the builder is released).
int stage_reserve(bsdb_builder *b, size_t bytes) {
    if (bytes <= b->stage_cap) return BSDB_OK;
    (void)hipFree(b->d_stage);
    b->d_stage = nullptr;
    b->stage_cap = 0;
    if (dmalloc(&b->d_stage, bytes) != hipSuccess) return BSDB_ENOMEM;
    b->stage_cap = bytes;
    return BSDB_OK;
}

// count device signatures (at the stage's front) with add positions pos0..:
// grouped by segment on the device, then appended to the host segments
// (caller holds the builder and context locks, device set)
int spill_segments(bsdb_builder *b, const ulonglong2 *d_sig, uint64_t count, uint64_t pos0, uint8_t *scr, hipStream_t s) {
    bsdb_ctx *c = b->c;
    uint32_t *d_cnt = (uint32_t *)scr;
    unsigned long long *d_cur = (unsigned long long *)(scr + 1024);
    ulonglong2 *o_sig = (ulonglong2 *)(scr + 1024 + 2048);
    uint64_t *o_pos = (uint64_t *)(o_sig + count);
    HIP_OK(hipMemsetAsync(d_cnt, 0, NSEG * 4, s));
    const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((count + SEG_CHUNK - 1) / SEG_CHUNK, (uint64_t)c->num_cus * 4));
    k_seg_count<<<g, 256, 0, s>>>(d_sig, count, d_cnt);
    uint32_t cnt[NSEG];
    unsigned long long base[NSEG];
    HIP_OK(hipMemcpyAsync(cnt, d_cnt, sizeof(cnt), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    unsigned long long run = 0;
    for (uint32_t k = 0; k < NSEG; ++k) {
        base[k] = run;
        run += cnt[k];
    }
    if (run != count) return BSDB_EIO;
    HIP_OK(hipMemcpyAsync(d_cur, base, sizeof(base), hipMemcpyHostToDevice, s));
    k_seg_scatter<<<g, 256, 0, s>>>(d_sig, count, pos0, d_cur, o_sig, o_pos);
    int rc = launch_status();
    if (rc) return rc;
    HIP_OK(hipStreamSynchronize(s));
    for (uint32_t k = 0; k < NSEG; ++k) {
        if (!cnt[k]) continue;
        HostVec<ulonglong2> &vs = b->seg_sig[k];
        HostVec<uint64_t> &vp = b->seg_pos[k];
        if (!vs.reserve(vs.n + cnt[k]) || !vp.reserve(vp.n + cnt[k])) return BSDB_ENOMEM;
        HIP_OK(hipMemcpyAsync(vs.p + vs.n, o_sig + base[k], (size_t)cnt[k] * 16, hipMemcpyDeviceToHost, s));
        HIP_OK(hipMemcpyAsync(vp.p + vp.n, o_pos + base[k], (size_t)cnt[k] * 8, hipMemcpyDeviceToHost, s));
        vs.n += cnt[k];
        vp.n += cnt[k];
    }
    HIP_OK(hipStreamSynchronize(s));
    return BSDB_OK;
}

// stage bytes for k keys of a spill round: signatures + the segment scratch
size_t spill_scratch_bytes(uint64_t k) { return 1024 + 2048 + (size_t)k * (16 + 16 + 8) + 256; }

void builder_drop_dev_records(bsdb_builder *b) {
    for (void **q : {&b->d_raddr, &b->d_rv8, &b->d_rvl}) {
        (void)hipFree(*q);
        *q = nullptr;
    }
    b->raddr_cap = b->rv8_cap = b->rvl_cap = 0;
    b->dev_rec = false;
}

// Switches a builder to spill mode: every resident key hashed on the device
// and moved to the host segments (its add position = its index), the key
// area released.  Caller holds mu, grow_mu exclusively (no copy in flight),
// the context lock, device set.
int builder_to_spill(bsdb_builder *b) {
    bsdb_ctx *c = b->c;
    hipStream_t s = c->stream;
    const uint64_t n = b->n;
    uint64_t chunk = 1ull << 24;  // keys a round (a multiple of 16: 16-B aligned fixed-length rounds)
    while (chunk >= 4096 && stage_reserve(b, spill_scratch_bytes(chunk) + chunk * 16))
        chunk >>= 1;
    if (chunk < 4096) return BSDB_ENOMEM;
    uint8_t *stage = (uint8_t *)b->d_stage;
    for (uint64_t k0 = 0; k0 < n; k0 += chunk) {
        const uint64_t k = std::min(chunk, n - k0);
        ulonglong2 *d_sig = (ulonglong2 *)stage;
        int rc = b->key_len ? hash_impl(c, b->d_keys + k0 * b->key_len, nullptr, k * b->key_len, b->key_len, k, 0,
                                        (uint64_t *)d_sig, s)
                            : hash_impl(c, b->d_keys, b->d_off + k0, b->key_bytes, 0, k, 0, (uint64_t *)d_sig, s);
        if (!rc) rc = spill_segments(b, d_sig, k, k0, stage + (size_t)chunk * 16, s);
        if (rc) return rc;
    }
    HIP_OK(hipStreamSynchronize(s));
    (void)hipFree(b->d_keys);
    (void)hipFree(b->d_off);
    b->d_keys = nullptr;
    b->d_off = nullptr;
    b->keys_cap = b->off_cap = 0;
    builder_drop_dev_records(b);  // (spill adds keep their records in host memory only)
    b->spill = true;
    if (getenv("BSDB_BUILDER_PROFILE"))
        fprintf(stderr, "[bsdb builder] spill mode after %llu keys (%llu key bytes)\n", (unsigned long long)n,
                (unsigned long long)b->key_bytes);
    return BSDB_OK;
}

// An add in spill mode (caller holds mu): the batch hashed on the device in
// rounds and appended to the host segments with positions n0..
int spill_add_locked(bsdb_builder *b, const AddBatch &a, uint64_t n0) {
    bsdb_ctx *c = b->c;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    hipStream_t s = c->stream;
    constexpr uint64_t ROUND_KEYS = 1ull << 23, ROUND_BYTES = 512ull << 20;
    for (uint64_t i0 = 0; i0 < a.count;) {
        uint64_t i1 = std::min(a.count, i0 + ROUND_KEYS);
        if (a.off)
            while (i1 - i0 > 1 && a.off[i1] - a.off[i0] > ROUND_BYTES) i1 = i0 + (i1 - i0) / 2;
        else
            i1 = std::min(i1, i0 + std::max<uint64_t>(1, ROUND_BYTES / a.key_len));
        const uint64_t k = i1 - i0;
        const uint64_t kbytes = a.off ? a.off[i1] - a.off[i0] : k * a.key_len;
        const size_t key_room = ((size_t)kbytes + 16 + 255) & ~(size_t)255, off_room = a.off ? ((k + 1) * 8 + 255) & ~(size_t)255 : 0;
        int rc = stage_reserve(b, key_room + off_room + (size_t)k * 16 + spill_scratch_bytes(k));
        if (rc) return rc;
        uint8_t *d_k = (uint8_t *)b->d_stage;
        uint64_t *d_o = (uint64_t *)(d_k + key_room);
        ulonglong2 *d_sig = (ulonglong2 *)(d_k + key_room + off_room);
        if (kbytes) HIP_OK(hipMemcpyAsync(d_k, a.off ? a.keys + a.off[i0] : a.keys + i0 * a.key_len, kbytes, hipMemcpyHostToDevice, s));
        if (a.off) {
            HIP_OK(hipMemcpyAsync(d_o, a.off + i0, (k + 1) * 8, hipMemcpyHostToDevice, s));
            k_rebase_offsets<<<grid_for(c, k + 1), 256, 0, s>>>(d_o, k + 1, (uint64_t)0 - a.off[i0]);
        }
        rc = a.off ? hash_impl(c, d_k, d_o, kbytes, 0, k, 0, (uint64_t *)d_sig, s)
                   : hash_impl(c, d_k, nullptr, kbytes, a.key_len, k, 0, (uint64_t *)d_sig, s);
        if (!rc) rc = spill_segments(b, d_sig, k, n0 + i0, (uint8_t *)(d_sig + k), s);
        if (rc) return rc;
        i0 = i1;
    }
    return BSDB_OK;
}

// Room for an add of `count` keys and `bytes` key bytes past the reserved
// ranges (caller holds mu).  A growth waits for the copies in flight
// (grow_mu exclusive); a key area that cannot grow (the device's HBM, or
// dev_key_cap) switches the builder to spill mode.
int builder_make_room(bsdb_builder *b, uint64_t count, uint64_t bytes) {
    const uint64_t n1 = b->n + count;
    const bool gh = !b->borrowed_records &&
                    ((!b->stride && n1 > b->addr.cap) || (b->approx && (n1 > b->value8.cap || n1 > b->vlen.cap)));
    const bool gk = !b->spill && (b->key_bytes + bytes + 16 > b->keys_cap || (!b->key_len && (n1 + 1) * 8 > b->off_cap));
    if (!gh && !gk) return BSDB_OK;
    std::unique_lock<std::shared_mutex> ex(b->grow_mu);
    bsdb_ctx *c = b->c;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    if (gh) {
        b->stop_prefault();  // (a growing array may move)
        if ((!b->stride && !b->addr.reserve(n1)) || (b->approx && (!b->value8.reserve(n1) || !b->vlen.reserve(n1))))
            return BSDB_ENOMEM;
        if (b->dev_rec && (dev_reserve(c, &b->d_raddr, &b->raddr_cap, b->n * 8, b->addr.cap * 8) ||
                           (b->approx && (dev_reserve(c, &b->d_rv8, &b->rv8_cap, b->n * 8, b->value8.cap * 8) ||
                                          dev_reserve(c, &b->d_rvl, &b->rvl_cap, b->n, b->vlen.cap))))) {
            builder_drop_dev_records(b);  // (the finish uploads them from host memory instead)
        }
    }
    if (!gk) return BSDB_OK;
    const uint64_t want = b->key_bytes + bytes + 16;
    int rc = want > b->dev_key_cap ? BSDB_ENOMEM
                                   : dev_reserve(c, (void **)&b->d_keys, &b->keys_cap, b->key_bytes, want, b->dev_key_cap);
    if (!rc && !b->key_len) rc = dev_reserve(c, (void **)&b->d_off, &b->off_cap, (b->n + 1) * 8, (n1 + 1) * 8);
    if (rc == BSDB_ENOMEM) rc = builder_to_spill(b);
    return rc;
}

// The batch's keys (and offsets) into the key area at key index n0 / key byte
// kb0, on a stream of the calling thread's own: adds run concurrently.
int add_copy_device(bsdb_builder *b, const AddBatch &a, uint64_t n0, uint64_t kb0, const uint64_t *h_addr,
                    const uint64_t *h_value8, const uint8_t *h_vlen) {
    bsdb_ctx *c = b->c;
    hipStream_t s = nullptr;
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    const uint64_t bytes = a.bytes();
    // one add alone: the runtime's pageable copy (56 GB/s for C4's 4 GiB
    // batches); several at once: each through pinned pieces
    const bool bounce = b->copying.fetch_add(1) > 0;
    // (BSDB_ADD_COPY=register, measurement: the source pinned in place for
    // its copy instead of the pinned pieces)
    static const bool reg_copy = getenv("BSDB_ADD_COPY") && !strcmp(getenv("BSDB_ADD_COPY"), "register");
    auto h2d = [&](void *dst, const void *src, size_t len) -> hipError_t {
        if (!len || e != hipSuccess) return e;
        if (bounce && reg_copy) {
            hipError_t r = hipHostRegister(const_cast<void *>(src), len, hipHostRegisterDefault);
            if (r != hipSuccess) return h2d_bounce(s, dst, src, len) ? hipErrorUnknown : hipSuccess;
            r = hipMemcpyAsync(dst, src, len, hipMemcpyHostToDevice, s);
            if (r == hipSuccess) r = hipStreamSynchronize(s);
            const hipError_t u = hipHostUnregister(const_cast<void *>(src));
            return r != hipSuccess ? r : u;
        }
        if (bounce) return h2d_bounce(s, dst, src, len) ? hipErrorUnknown : hipSuccess;
        return hipMemcpyAsync(dst, src, len, hipMemcpyHostToDevice, s);
    };
    e = h2d(b->d_keys + kb0, a.first(), bytes);
    if (b->dev_rec && !b->borrowed_records && a.count) {
        if (!b->stride) e = h2d((uint64_t *)b->d_raddr + n0, h_addr, a.count * 8);
        if (b->approx) {
            e = h2d((uint64_t *)b->d_rv8 + n0, h_value8, a.count * 8);
            e = h2d((uint8_t *)b->d_rvl + n0, h_vlen, a.count);
        }
    }
    if (e == hipSuccess && !b->key_len && a.count) {  // a variable-length builder's offsets
        uint64_t *dst = b->d_off + n0 + 1;
        if (a.uni != 0xFFFFFFFFu) {
            // one length (a kv.db partition of fixed-size keys): the offsets
            // are a formula, written on the device instead of copied
            k_fill_offsets<<<grid_for(c, a.count), 256, 0, s>>>(dst, a.count, kb0, a.uni);
            e = hipGetLastError();
        } else {
            e = hipMemcpyAsync(dst, a.off + 1, a.count * 8, hipMemcpyHostToDevice, s);
            if (e == hipSuccess) {
                k_rebase_offsets<<<grid_for(c, a.count), 256, 0, s>>>(dst, a.count, kb0 - a.o0());
                e = hipGetLastError();
            }
        }
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);  // the caller may reuse its buffers
    if (s) (void)hipStreamDestroy(s);
    b->copying.fetch_sub(1);
    return e == hipSuccess ? BSDB_OK : hip_fail(e, "builder add copy", __LINE__);
}

void add_copy_records(bsdb_builder *b, uint64_t n0, uint64_t count, const uint64_t *h_addr, const uint64_t *h_value8,
                      const uint8_t *h_vlen) {
    if (b->borrowed_records || !count) return;
    if (!b->stride) memcpy(b->addr.p + n0, h_addr, count * 8);
    if (b->approx) {
        memcpy(b->value8.p + n0, h_value8, count * 8);
        memcpy(b->vlen.p + n0, h_vlen, count);
    }
}

// One add: its ranges reserved under the builder's lock, the copies outside
// it (concurrently with other adds); a failure marks the builder failed.
int builder_add(bsdb_builder *b, const AddBatch &a, const uint64_t *h_addr, const uint64_t *h_value8,
                const uint8_t *h_vlen) {
    std::shared_lock<std::shared_mutex> copying;
    uint64_t n0 = 0, kb0 = 0;
    {
        std::lock_guard<std::mutex> gb(b->mu);
        if (b->failed) return b->failed;
        if (b->finished) return BSDB_EINVAL;
        int rc = builder_check_records(b, a.count, h_addr, h_value8, h_vlen);
        if (rc) return rc;
        if (a.count == 0) return BSDB_OK;
        const uint64_t bytes = a.bytes();
        if ((rc = builder_make_room(b, a.count, bytes))) return b->failed = rc;
        n0 = b->n;
        kb0 = b->key_bytes;
        if (!b->key_len) {
            const uint32_t len = a.off ? a.uni : a.key_len;
            if (n0 == 0) b->uni_len = len;
            b->uniform = b->uniform && len != 0xFFFFFFFFu && len == b->uni_len;
        }
        if (b->spill) {
            // (serialised: the device hash and the segment appends)
            if ((rc = spill_add_locked(b, a, n0))) return b->failed = rc;
            add_copy_records(b, n0, a.count, h_addr, h_value8, h_vlen);
        } else {
            copying = std::shared_lock<std::shared_mutex>(b->grow_mu);  // (before mu is released: no growth between)
        }
        b->n += a.count;
        b->key_bytes += bytes;
        if (!b->borrowed_records) {
            if (!b->stride) b->addr.n = b->n;
            if (b->approx) b->value8.n = b->vlen.n = b->n;
        }
        if (b->spill) return BSDB_OK;
    }
    const auto t0 = std::chrono::steady_clock::now();
    int rc = add_copy_device(b, a, n0, kb0, h_addr, h_value8, h_vlen);
    const auto t1 = std::chrono::steady_clock::now();
    add_copy_records(b, n0, a.count, h_addr, h_value8, h_vlen);
    b->add_copy_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    b->add_rec_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t1).count();
    if (rc) {
        int expect = BSDB_OK;
        b->copy_failed.compare_exchange_strong(expect, rc);
    }
    copying.unlock();
    if (rc) {
        std::lock_guard<std::mutex> gb(b->mu);
        if (!b->failed) b->failed = rc;
    }
    return rc;
}

// creates (truncates) an index file at its final size and maps a regular
// file for the writer threads; a path that is not a regular file (e.g.
// /dev/null for a measurement without a file system) is written with pwrite
int open_out(const char *path, uint64_t bytes, OutFile *o) {
    o->fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
    if (o->fd < 0) o->fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);  // (e.g. a write-only device)
    if (o->fd < 0) return BSDB_EFILE;
    struct stat st;
    if (fstat(o->fd, &st) != 0) return BSDB_EFILE;
    if (!S_ISREG(st.st_mode) || !bytes) return BSDB_OK;
    if (ftruncate(o->fd, (off_t)bytes) != 0) return BSDB_EFILE;
    // mapped only where blocks can be reserved ahead of the stores (a file
    // system without fallocate is written with pwrite, which reports ENOSPC)
    const int res = file_reserve(o->fd, 0, std::min<uint64_t>(bytes, 1u << 16));
    if (res < 0) return BSDB_EFILE;
    void *m = getenv("BSDB_NO_MMAP_WRITE") || res ? MAP_FAILED
                                                   : mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, o->fd, 0);
    if (m != MAP_FAILED) {
        o->map = (uint8_t *)m;
        o->bytes = bytes;
    }
    return BSDB_OK;
}

int close_out(OutFile &o) {
    bool ok = true;
    if (o.map) ok = munmap(o.map, o.bytes) == 0;
    if (o.fd >= 0) ok = close(o.fd) == 0 && ok;
    o = OutFile{};
    return ok ? BSDB_OK : BSDB_EFILE;
}

// The build of everything added so far (caller holds the context lock).
int builder_finish_locked(bsdb_builder *b, uint32_t width, uint32_t passes, const char *index_path,
                          const char *index_a_path, bsdb_mph **out, uint32_t *passes_used) {
    bsdb_ctx *c = b->c;
    const uint64_t n = b->n;
    OutFile fo, fao;
    Populator pop_o, pop_a;
    void *d_addr = nullptr, *d_v8 = nullptr, *d_vl = nullptr;
    void *slot_a[2] = {nullptr, nullptr};
    size_t slot_a_bytes[2] = {0, 0};
    void *sp_in = nullptr, *sp_out = nullptr;  // spill mode: a pass's uploaded segments, its compacted keys
    size_t sp_in_bytes = 0, sp_out_bytes = 0;
    bsdb_mph *p = nullptr;
    std::thread host_rel;  // the host record arrays' release, once the device copies took over
    // BSDB_BUILDER_PROFILE=1: the finish's phases on stderr
    const bool prof = getenv("BSDB_BUILDER_PROFILE") != nullptr;
    const auto t_start = std::chrono::steady_clock::now();
    auto mark = [&](const char *what) {
        if (prof)
            fprintf(stderr, "[bsdb builder] finish %s at %.3f s\n", what,
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count());
    };
    auto done = [&](int rc) {
        if (b->on_opened) b->on_opened();  // (every exit releases the caller's hold)
        b->on_opened = nullptr;
        (void)hipStreamSynchronize(c->stream);
        if (host_rel.joinable()) host_rel.join();
        for (void *q : {d_addr, d_v8, d_vl, slot_a[0], slot_a[1], sp_in, sp_out}) (void)hipFree(q);
        pop_o.finish();
        pop_a.finish();
        if (prof && fo.map)
            fprintf(stderr, "[bsdb builder] index pages prefaulted in %.3f s (index_a %.3f s)\n", pop_o.seconds, pop_a.seconds);
        mark("buffers released");
        if (close_out(fo) && !rc) rc = BSDB_EFILE;
        if (close_out(fao) && !rc) rc = BSDB_EFILE;
        mark("files closed");
        if (rc && p) mph_release(p);
        if (!rc) *out = p;
        return rc;
    };
    // (every failure from here on goes through done(): the files, their
    // populators, the device buffers and the MPHF are released)
#define FIN_OK(x)                                                         \
    do {                                                                  \
        const hipError_t e_ = (x);                                        \
        if (e_ != hipSuccess) return done(hip_fail(e_, #x, __LINE__));    \
    } while (0)
    // W:124-127: both files created first; index_a.db stays empty in exact mode
    int rc = BSDB_OK;
    if (index_path && ((rc = open_out(index_path, n * 8, &fo)) ||
                       (index_a_path && (rc = open_out(index_a_path, b->approx ? n * 8 : 0, &fao)))))
        return done(rc);
    mark("index file created");
    // (the device arrays before the populators start: an allocation maps
    // into the address space, which each populate step holds)
    if ((rc = mph_alloc(c, n, width, &p))) return done(rc);
    pop_o.start(fo.map, fo.bytes, fo.fd, 0);
    pop_a.start(fao.map, fao.bytes, fao.fd, 0);
    fo.pop = &pop_o;
    fao.pop = &pop_a;
    mark("files opened");
    if (b->on_opened) b->on_opened();
    b->on_opened = nullptr;
    if (prof)
        fprintf(stderr, "[bsdb builder] adds: device copies %.3f s, record copies %.3f s (thread totals)%s\n",
                b->add_copy_ns.load() / 1e9, b->add_rec_ns.load() / 1e9, b->dev_rec ? ", records on the device" : "");
    if (n == 0) {  // E = {0}, no values beyond the trailing word (GOV:484)
        FIN_OK(hipMemsetAsync(p->E, 0, (p->m + 1) * 8, c->stream));
        FIN_OK(hipMemsetAsync(p->values, 0, p->values_words * 8, c->stream));
        if (width) FIN_OK(hipMemsetAsync(p->sigbits, 0, p->sig_words * 8, c->stream));
        return done(BSDB_OK);
    }
    GovSrc src;
    src.n = n;
    src.keys = b->d_keys;
    const uint32_t flen = b->key_len ? b->key_len : (b->uniform && !bad_key_len(b->uni_len) ? b->uni_len : 0);
    if (flen) {  // every key has one length: the fixed-length kernels over the same bytes
        src.key_len = flen;
        src.blob_bytes = n * flen;
    } else {
        src.off = b->d_off;
        src.blob_bytes = b->key_bytes;
    }
    PassSink sink;
    const uint64_t *dev_addr = nullptr;
    if (index_path) {
        // where the addresses (and value bytes) are read: HBM if they fit in a
        // quarter of what the keys left free, else host memory
        size_t free_b = 0, total_b = 0;
        FIN_OK(hipMemGetInfo(&free_b, &total_b));
        const uint64_t rec_bytes = n * ((b->stride ? 0 : 8) + (b->approx ? 9 : 0));
        const bool host_gather = getenv("BSDB_BUILDER_HOST_GATHER") != nullptr || (!b->dev_rec && rec_bytes > free_b / 4);
        if (!host_gather && b->dev_rec) {
            // uploaded by the adds: the finish takes them over
            d_addr = b->d_raddr;
            d_v8 = b->d_rv8;
            d_vl = b->d_rvl;
            b->d_raddr = b->d_rv8 = b->d_rvl = nullptr;
            b->raddr_cap = b->rv8_cap = b->rvl_cap = 0;
            b->dev_rec = false;
            dev_addr = (const uint64_t *)d_addr;
            // the host copies are dead: released beside the passes (a 1e8-key
            // build's 800 MB took ~45 ms after them)
            host_rel = std::thread([b] {
                b->stop_prefault();
                b->addr.release();
                b->value8.release();
                b->vlen.release();
            });
        } else if (!host_gather) {
            const int dev = c->device;
            int up_rc = BSDB_OK;
            if (!b->stride && (dmalloc(&d_addr, n * 8) != hipSuccess || (up_rc = h2d_pageable(dev, d_addr, b->addr.p, n * 8))))
                return done(up_rc ? up_rc : BSDB_ENOMEM);
            if (b->approx && (dmalloc(&d_v8, n * 8) != hipSuccess || dmalloc(&d_vl, n) != hipSuccess ||
                              (up_rc = h2d_pageable(dev, d_v8, b->value8.p, n * 8)) ||
                              (up_rc = h2d_pageable(dev, d_vl, b->vlen.p, n))))
                return done(up_rc ? up_rc : BSDB_ENOMEM);
            dev_addr = (const uint64_t *)d_addr;
        }
        if (!b->approx && !host_gather && !b->spill) {
            // the solve stores the final slots (addr[p] or base + stride p)
            sink.job = [&](int, const uint64_t *d_slice, uint64_t nl, uint64_t e_lo) {
                return write_slots(c->device, fo, d_slice, nl, e_lo, nullptr, nullptr);
            };
        } else if (!host_gather) {
            // approximate (or spill mode): positions in the slots, gathered on the device
            sink.positions = true;
            sink.job_bytes_per_key = b->approx ? 16 : 8;
            sink.prepare = [&](int sl, uint64_t nl) {
                return b->approx ? grow(&slot_a[sl], &slot_a_bytes[sl], std::max<uint64_t>(nl, 1) * 8) : BSDB_OK;
            };
            sink.job = [&](int sl, const uint64_t *d_slice, uint64_t nl, uint64_t e_lo) {
                hipStream_t st = nullptr;
                if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return BSDB_EIO;
                k_slot_gather<<<grid_for(c, nl), 256, 0, st>>>(const_cast<uint64_t *>(d_slice), nl, dev_addr,
                                                                b->addr_base, b->addr_stride, (const uint64_t *)d_v8,
                                                                (const uint8_t *)d_vl,
                                                                b->approx ? (uint64_t *)slot_a[sl] : nullptr);
                const bool ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
                (void)hipStreamDestroy(st);
                if (!ok) return BSDB_EIO;
                int r = write_slots(c->device, fo, d_slice, nl, e_lo, nullptr, nullptr);
                if (!r && b->approx) r = write_slots(c->device, fao, (const uint64_t *)slot_a[sl], nl, e_lo, nullptr, nullptr);
                return r;
            };
        } else {
            // positions in the slots, addresses gathered from host memory by
            // the writer threads
            sink.positions = true;
            const uint64_t *ha = b->addr.p, *hv = b->value8.p;
            const uint8_t *hl = b->vlen.p;
            const bool st = b->stride, ap = b->approx;
            const uint64_t base = b->addr_base, stride = b->addr_stride;
            const SlotXform xf = [=](uint64_t *piece, uint64_t k, uint64_t *piece_a) {
                for (uint64_t i = 0; i < k; ++i) {
                    const uint64_t q = __builtin_bswap64(piece[i]);
                    piece[i] = __builtin_bswap64(st ? base + stride * q : ha[q]);
                    if (ap && piece_a) {
                        const uint32_t l = hl[q] < 8 ? hl[q] : 8;
                        piece_a[i] = l >= 8 ? hv[q] : hv[q] & ((1ULL << (8 * l)) - 1);
                    }
                }
            };
            sink.job = [&, xf](int, const uint64_t *d_slice, uint64_t nl, uint64_t e_lo) {
                return write_slots(c->device, fo, d_slice, nl, e_lo, &xf, b->approx ? &fao : nullptr);
            };
        }
    }
    mark("records placed");
    if (b->spill) {
        // Spill mode: pass p's keys are those of the 256 host segments that
        // can hold its buckets [b_lo, b_hi) -- the segment is sig0's top byte
        // and the bucket is monotone in sig0 (CBHS:129-138, 900, 965), so a
        // contiguous run of segments, the two at its ends shared with the
        // neighbouring passes -- uploaded and compacted to the range on the
        // device; each key's add position goes into its slot (positions mode).
        const uint64_t mult = 2 * (n / BUCKET_SIZE + 1);
        sink.positions = true;
        sink.source_bytes_per_key = 2 * 24 + 8;
        sink.source = [&](uint64_t b_lo, uint64_t b_hi, GovSrc &ps, const uint64_t **pos) -> int {
            auto x_first = [&](uint64_t bk) { return (((unsigned __int128)bk << 64) + mult - 1) / mult; };  // first sig0 >>> 1 of bucket bk
            const uint32_t s_a = (uint32_t)(x_first(b_lo) >> 55), s_b = (uint32_t)((x_first(b_hi) - 1) >> 55);
            uint64_t tot = 0;
            for (uint32_t k = s_a; k <= s_b && k < NSEG; ++k) tot += b->seg_sig[k].n;
            int r;
            if ((r = grow(&sp_in, &sp_in_bytes, tot * 24 + 256)) || (r = grow(&sp_out, &sp_out_bytes, tot * 24 + 512)))
                return r;
            ulonglong2 *in_sig = (ulonglong2 *)sp_in, *out_sig = (ulonglong2 *)sp_out;
            uint64_t *in_pos = (uint64_t *)(in_sig + tot), *out_pos = (uint64_t *)(out_sig + tot);
            unsigned long long *d_cnt = (unsigned long long *)(out_pos + tot);
            hipStream_t st = c->stream;
            uint64_t at = 0;
            for (uint32_t k = s_a; k <= s_b && k < NSEG; ++k) {
                const uint64_t kn = b->seg_sig[k].n;
                if (!kn) continue;
                HIP_OK(hipMemcpyAsync(in_sig + at, b->seg_sig[k].p, kn * 16, hipMemcpyHostToDevice, st));
                HIP_OK(hipMemcpyAsync(in_pos + at, b->seg_pos[k].p, kn * 8, hipMemcpyHostToDevice, st));
                at += kn;
            }
            HIP_OK(hipMemsetAsync(d_cnt, 0, 8, st));
            if (tot)
                k_range_compact<<<grid_for(c, tot), 256, 0, st>>>(in_sig, in_pos, tot, (uint32_t)mult, (uint32_t)b_lo,
                                                                  (uint32_t)b_hi, out_sig, out_pos, d_cnt);
            if ((r = launch_status())) return r;
            unsigned long long got = 0;
            HIP_OK(hipMemcpyAsync(&got, d_cnt, 8, hipMemcpyDeviceToHost, st));
            HIP_OK(hipStreamSynchronize(st));
            ps = GovSrc{};
            ps.sig = tot ? (const uint64_t *)out_sig : reinterpret_cast<const uint64_t *>(16);  // (n == 0: never read)
            ps.n = got;
            *pos = out_pos;
            return BSDB_OK;
        };
    }
    rc = passes_build(c, src, n, width, passes, dev_addr, b->addr_base, b->addr_stride, p->E, p->values, p->sigbits,
                      sink, passes_used, c->stream);
    mark("passes done");
    return done(rc);
#undef FIN_OK
}

void builder_release(bsdb_builder *b) {
    const auto t0 = std::chrono::steady_clock::now();
    b->stop_prefault();
    (void)hipSetDevice(b->c->device);
    (void)hipFree(b->d_keys);
    (void)hipFree(b->d_off);
    (void)hipFree(b->d_stage);
    builder_drop_dev_records(b);
    if (getenv("BSDB_BUILDER_PROFILE"))
        fprintf(stderr, "[bsdb builder] release: prefault stopped, device freed in %.3f s\n",
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    b->d_keys = nullptr;
    b->d_off = nullptr;
    b->d_stage = nullptr;
    b->keys_cap = b->off_cap = b->stage_cap = 0;
    for (uint32_t k = 0; k < NSEG; ++k) {
        b->seg_sig[k].release();
        b->seg_pos[k].release();
    }
    b->addr.release();
    b->value8.release();
    b->vlen.release();
}

// borrowed: the caller's record arrays will be borrowed (host_passes_build):
// no host arrays reserved, no populator started
int builder_open(bsdb_ctx *c, uint32_t key_len, uint64_t key_capacity, uint64_t blob_capacity, int approximate,
                 uint64_t addr_base, uint64_t addr_stride, bsdb_builder **out, bool borrowed = false) {
    if (!c || !out || (key_len && bad_key_len(key_len))) return BSDB_EINVAL;
    *out = nullptr;
    bsdb_builder *b = new (std::nothrow) bsdb_builder();
    if (!b) return BSDB_ENOMEM;
    b->c = c;
    b->key_len = key_len;
    b->approx = approximate != 0;
    b->stride = addr_stride != 0;
    b->addr_base = addr_base;
    b->addr_stride = addr_stride;
    b->borrowed_records = borrowed;
    // BSDB_BUILDER_DEVICE_KEY_BYTES (a test knob): the most key bytes the
    // device key area may hold; adds past it switch to spill mode
    if (const char *v = getenv("BSDB_BUILDER_DEVICE_KEY_BYTES")) b->dev_key_cap = std::max<uint64_t>(4096, strtoull(v, nullptr, 0));
    int rc = BSDB_OK;
    {
        std::lock_guard<std::mutex> g(c->mu);
        if (hipSetDevice(c->device) != hipSuccess) {
            rc = BSDB_EIO;
        } else {
            Ordered ord(c, c->stream);
            const uint64_t kb = std::min<uint64_t>((key_len ? key_capacity * key_len : blob_capacity) + 16, b->dev_key_cap);
            rc = dev_reserve(c, (void **)&b->d_keys, &b->keys_cap, 0, kb);
            // (a capacity HBM cannot hold: a smaller area now, spill mode when the adds outgrow what HBM allows)
            if (rc == BSDB_ENOMEM && kb > (64ull << 20)) rc = dev_reserve(c, (void **)&b->d_keys, &b->keys_cap, 0, 64ull << 20);
            if (!rc && !key_len) {
                rc = dev_reserve(c, (void **)&b->d_off, &b->off_cap, 0, (key_capacity + 1) * 8);
                if (!rc && hipMemsetAsync(b->d_off, 0, 8, c->stream) != hipSuccess) rc = BSDB_EIO;
                if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = BSDB_EIO;
            }
        }
    }
    if (!rc && !borrowed &&
        ((!b->stride && !b->addr.reserve(key_capacity)) ||
         (b->approx && (!b->value8.reserve(key_capacity) || !b->vlen.reserve(key_capacity)))))
        rc = BSDB_ENOMEM;
    if (!rc && !borrowed && key_capacity && (!b->stride || b->approx)) {
        // the records on the device too, when they fit an eighth of the free HBM
        std::lock_guard<std::mutex> g(c->mu);
        size_t free_b = 0, total_b = 0;
        const uint64_t cap = b->stride ? b->value8.cap : b->addr.cap;
        const uint64_t want = cap * ((b->stride ? 0 : 8) + (b->approx ? 9 : 0));
        if (hipSetDevice(c->device) == hipSuccess && hipMemGetInfo(&free_b, &total_b) == hipSuccess && want <= free_b / 8) {
            b->dev_rec = (b->stride || dev_reserve(c, &b->d_raddr, &b->raddr_cap, 0, b->addr.cap * 8) == BSDB_OK) &&
                         (!b->approx || (dev_reserve(c, &b->d_rv8, &b->rv8_cap, 0, b->value8.cap * 8) == BSDB_OK &&
                                         dev_reserve(c, &b->d_rvl, &b->rvl_cap, 0, b->vlen.cap) == BSDB_OK));
            if (!b->dev_rec) builder_drop_dev_records(b);
        }
    }
    if (rc) {
        builder_release(b);
        delete b;
        return rc;
    }
    if (!borrowed && !b->stride && b->addr.cap) b->pop_addr.start(reinterpret_cast<uint8_t *>(b->addr.p), b->addr.cap * 8);
    if (!borrowed && b->approx && b->value8.cap) b->pop_v8.start(reinterpret_cast<uint8_t *>(b->value8.p), b->value8.cap * 8);
    *out = b;
    return BSDB_OK;
}

}  // namespace

// ---- one-call forms over host arrays (used by the F2 entry points when the
// one-shot build does not fit the device) ----------------------------------
static int host_passes_build(bsdb_ctx *c, const uint8_t *h_keys, uint32_t key_len, const uint8_t *h_blob,
                             const uint64_t *h_off, uint64_t n, uint32_t width, const uint64_t *h_addr,
                             uint64_t addr_base, uint64_t addr_stride, const uint64_t *h_value8, const uint8_t *h_vlen,
                             int approximate, uint32_t passes, const char *index_path, const char *index_a_path,
                             bsdb_mph **out, uint32_t *passes_used) {
    const bool var = h_off != nullptr;
    const uint64_t blob = var ? (n ? h_off[n] - h_off[0] : 0) : 0;
    bsdb_builder *b = nullptr;
    int rc = builder_open(c, var ? 0 : key_len, n, blob, approximate, addr_base, h_addr ? 0 : addr_stride, &b, true);
    if (rc) return rc;
    // the caller's record arrays outlive the call: borrowed, not copied
    if (h_addr) b->addr.borrow(h_addr, n);
    if (approximate) {
        b->value8.borrow(h_value8, n);
        b->vlen.borrow(h_vlen, n);
    }
    // keys in batches of <= 4 GiB (one synchronous copy each)
    constexpr uint64_t BATCH = 4ULL << 30;
    for (uint64_t k0 = 0; k0 < n && !rc;) {
        uint64_t k1;
        if (var) {
            k1 = std::min<uint64_t>(n, k0 + (1ULL << 28));
            while (k1 - k0 > 1 && h_off[k1] - h_off[k0] > BATCH) k1 = k0 + (k1 - k0) / 2;
            uint32_t uni = 0;
            rc = var_batch_lengths(h_off + k0, k1 - k0, &uni);
            AddBatch a;
            a.keys = h_blob;
            a.off = h_off + k0;
            a.count = k1 - k0;
            a.uni = uni;
            if (!rc) rc = builder_add(b, a, nullptr, nullptr, nullptr);
        } else {
            k1 = std::min(n, k0 + std::max<uint64_t>(1, BATCH / key_len));
            AddBatch a;
            a.keys = h_keys + k0 * key_len;
            a.key_len = a.uni = key_len;
            a.count = k1 - k0;
            rc = builder_add(b, a, nullptr, nullptr, nullptr);
        }
        k0 = k1;
    }
    if (!rc) {
        std::lock_guard<std::mutex> gb(b->mu);
        std::unique_lock<std::shared_mutex> settled(b->grow_mu);
        std::lock_guard<std::mutex> g(c->mu);
        if (b->copy_failed.load()) {
            rc = b->failed = b->copy_failed.load();
        } else if (hipSetDevice(c->device) != hipSuccess) {
            rc = BSDB_EIO;
        } else {
            Ordered ord(c, c->stream);
            rc = builder_finish_locked(b, width, passes, index_path, index_a_path, out, passes_used);
            builder_release(b);
        }
    } else {
        builder_release(b);
    }
    delete b;
    return rc;
}

// Whether the one-shot F2 build (bsdb_mph_build_index_*: signatures, their
// sorted copy, positions, ranks, addresses and the whole index on the device
// at once) fits the free HBM; otherwise those entry points take the passes.
static bool one_shot_fits(bsdb_ctx *c, uint64_t n, bool approx) {
    size_t free_b = 0, total_b = 0;
    {
        std::lock_guard<std::mutex> g(c->mu);
        if (hipSetDevice(c->device) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess) return true;
    }
    const double per_key = 16 + 16 + 8 + 8 + 8 + 8 + (approx ? 17 : 0) + 1.5;
    return (double)n * per_key * 1.05 + 12e9 < 0.9 * (double)free_b;
}

extern "C" {

int bsdb_builder_open(bsdb_ctx *c, uint32_t key_len, uint64_t key_capacity, uint64_t blob_capacity, int approximate,
                      uint64_t addr_base, uint64_t addr_stride, bsdb_builder **out) {
    return builder_open(c, key_len, key_capacity, blob_capacity, approximate, addr_base, addr_stride, out);
}

int bsdb_builder_add_fixed(bsdb_builder *b, const uint8_t *h_keys, uint32_t key_len, uint64_t count,
                           const uint64_t *h_addr, const uint64_t *h_value8, const uint8_t *h_vlen) {
    if (!b || bad_key_len(key_len) || (count && !h_keys) || (b->key_len && key_len != b->key_len)) return BSDB_EINVAL;
    AddBatch a;
    a.keys = h_keys;
    a.key_len = a.uni = key_len;
    a.count = count;
    return builder_add(b, a, h_addr, h_value8, h_vlen);
}

int bsdb_builder_add_var(bsdb_builder *b, const uint8_t *h_blob, const uint64_t *h_off, uint64_t count,
                         const uint64_t *h_addr, const uint64_t *h_value8, const uint8_t *h_vlen) {
    if (!b || b->key_len || (count && (!h_blob || !h_off))) return BSDB_EINVAL;
    uint32_t uni = 0;
    if (count && var_batch_lengths(h_off, count, &uni)) return BSDB_EINVAL;
    AddBatch a;
    a.keys = h_blob;
    a.off = h_off;
    a.count = count;
    a.uni = uni;
    return builder_add(b, a, h_addr, h_value8, h_vlen);
}

int bsdb_builder_count(const bsdb_builder *b, uint64_t *n) {
    if (!b || !n) return BSDB_EINVAL;
    std::lock_guard<std::mutex> gb(const_cast<bsdb_builder *>(b)->mu);  // (adds reserve under it: ADVICE r4)
    *n = b->n;
    return BSDB_OK;
}

int bsdb_builder_finish(bsdb_builder *b, uint32_t width, uint32_t passes, const char *index_path,
                        const char *index_a_path, bsdb_mph **out, uint32_t *passes_used) {
    if (!b || !out || width > 64 || passes > 4096 || (b->approx && index_path && !index_a_path)) return BSDB_EINVAL;
    *out = nullptr;
    std::lock_guard<std::mutex> gb(b->mu);
    if (b->failed) return b->failed;
    if (b->finished || b->n / BUCKET_SIZE + 1 > 0x7FFFFFFFULL) return BSDB_EINVAL;
    bsdb_ctx *c = b->c;
    int rc;
    {
        std::unique_lock<std::shared_mutex> settled(b->grow_mu);  // every add's copies are done
        if (const int cf = b->copy_failed.load()) return b->failed = cf;  // a copy failed after the check above
        std::lock_guard<std::mutex> g(c->mu);
        HIP_OK(hipSetDevice(c->device));
        Ordered ord(c, c->stream);
        rc = builder_finish_locked(b, width, passes, index_path, index_a_path, out, passes_used);
        b->finished = true;
        const auto t_rel = std::chrono::steady_clock::now();
        builder_release(b);  // the keys leave HBM: the MPHF stays
        if (getenv("BSDB_BUILDER_PROFILE"))
            fprintf(stderr, "[bsdb builder] builder released in %.3f s\n",
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t_rel).count());
    }
    return rc;
}

int bsdb_builder_free(bsdb_builder *b) {
    if (!b) return BSDB_EINVAL;
    {
        std::lock_guard<std::mutex> g(b->c->mu);
        (void)hipSetDevice(b->c->device);
        (void)hipStreamSynchronize(b->c->stream);
        builder_release(b);
    }
    delete b;
    return BSDB_OK;
}

int bsdb_mph_build_index_passes_fixed(bsdb_ctx *c, const uint8_t *h_keys, uint32_t key_len, uint64_t n,
                                      uint32_t width, const uint64_t *h_addr, uint64_t addr_base, uint64_t addr_stride,
                                      const uint64_t *h_value8, const uint8_t *h_vlen, int approximate, uint32_t passes,
                                      const char *index_path, const char *index_a_path, bsdb_mph **out,
                                      uint32_t *passes_used) {
    if (!c || !out || !index_path || bad_key_len(key_len) || width > 64 || passes > 4096 ||
        (approximate && !index_a_path) ||
        (n && (!h_keys || (!h_addr && !addr_stride) || (approximate && (!h_value8 || !h_vlen)))) ||
        n / BUCKET_SIZE + 1 > 0x7FFFFFFFULL)
        return BSDB_EINVAL;
    *out = nullptr;
    return host_passes_build(c, h_keys, key_len, nullptr, nullptr, n, width, h_addr, addr_base, addr_stride, h_value8,
                             h_vlen, approximate, passes, index_path, index_a_path, out, passes_used);
}

int bsdb_mph_build_index_passes_var(bsdb_ctx *c, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n,
                                    uint32_t width, const uint64_t *h_addr, uint64_t addr_base, uint64_t addr_stride,
                                    const uint64_t *h_value8, const uint8_t *h_vlen, int approximate, uint32_t passes,
                                    const char *index_path, const char *index_a_path, bsdb_mph **out,
                                    uint32_t *passes_used) {
    if (!c || !out || !index_path || width > 64 || passes > 4096 || (approximate && !index_a_path) || !h_off ||
        (n && (!h_blob || (!h_addr && !addr_stride) || (approximate && (!h_value8 || !h_vlen)))) ||
        n / BUCKET_SIZE + 1 > 0x7FFFFFFFULL)
        return BSDB_EINVAL;
    *out = nullptr;
    return host_passes_build(c, nullptr, 0, h_blob, h_off, n, width, h_addr, addr_base, addr_stride, h_value8, h_vlen,
                             approximate, passes, index_path, index_a_path, out, passes_used);
}

}  // extern "C"

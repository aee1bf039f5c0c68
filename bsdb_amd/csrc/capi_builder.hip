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
    bool finished = false;
    std::mutex mu;  // one add (or the finish) at a time: adds may come from several threads
    // the record arrays' pages, populated in the background from the open
    // (first-touch faults of ~2 µs a page were most of an add's time)
    Populator pop_addr, pop_v8;
    void stop_prefault() {
        pop_addr.finish();
        pop_v8.finish();
    }
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
int dev_reserve(bsdb_ctx *c, void **p, size_t *cap, size_t used, size_t need) {
    if (need <= *cap) return BSDB_OK;
    void *q = nullptr;
    size_t nc = std::max(need, *cap + *cap / 2);
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

int builder_add_records(bsdb_builder *b, uint64_t count, const uint64_t *h_addr, const uint64_t *h_value8,
                        const uint8_t *h_vlen) {
    if (b->borrowed_records) return BSDB_OK;
    if ((!b->stride && b->addr.n + count > b->addr.cap) || (b->approx && b->value8.n + count > b->value8.cap))
        b->stop_prefault();  // (a growing array may move)
    if (!b->stride && !b->addr.append(h_addr, count)) return BSDB_ENOMEM;
    if (b->approx && (!b->value8.append(h_value8, count) || !b->vlen.append(h_vlen, count))) return BSDB_ENOMEM;
    return BSDB_OK;
}

// one add of fixed-length keys (caller holds the context lock, device set)
int builder_add_fixed_locked(bsdb_builder *b, const uint8_t *h_keys, uint32_t key_len, uint64_t count) {
    bsdb_ctx *c = b->c;
    const uint64_t bytes = (uint64_t)key_len * count;
    int rc = dev_reserve(c, (void **)&b->d_keys, &b->keys_cap, b->key_bytes, b->key_bytes + bytes + 16);
    if (rc) return rc;
    if (bytes) HIP_OK(hipMemcpyAsync(b->d_keys + b->key_bytes, h_keys, bytes, hipMemcpyHostToDevice, c->stream));
    if (!b->key_len) {  // a variable-length builder: offsets key_bytes + (i + 1) L
        if ((rc = dev_reserve(c, (void **)&b->d_off, &b->off_cap, (b->n + 1) * 8, (b->n + count + 1) * 8))) return rc;
        if (count)
            k_fill_offsets<<<grid_for(c, count), 256, 0, c->stream>>>(b->d_off + b->n + 1, count, b->key_bytes,
                                                                      key_len);
        if (b->n == 0) b->uni_len = key_len;
        b->uniform = b->uniform && key_len == b->uni_len;
    }
    HIP_OK(hipStreamSynchronize(c->stream));  // the caller may reuse its buffers
    if ((rc = launch_status())) return rc;
    b->key_bytes += bytes;
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

// one add of variable-length keys whose lengths var_batch_lengths has
// checked (uni: their common length or 0xFFFFFFFF)
int builder_add_var_locked(bsdb_builder *b, const uint8_t *h_blob, const uint64_t *h_off, uint64_t count,
                           uint32_t uni) {
    bsdb_ctx *c = b->c;
    if (count == 0) return BSDB_OK;
    const uint64_t o0 = h_off[0], bytes = h_off[count] - o0;
    int rc = dev_reserve(c, (void **)&b->d_keys, &b->keys_cap, b->key_bytes, b->key_bytes + bytes + 16);
    if (rc) return rc;
    if ((rc = dev_reserve(c, (void **)&b->d_off, &b->off_cap, (b->n + 1) * 8, (b->n + count + 1) * 8))) return rc;
    if (bytes) HIP_OK(hipMemcpyAsync(b->d_keys + b->key_bytes, h_blob + o0, bytes, hipMemcpyHostToDevice, c->stream));
    uint64_t *dst = b->d_off + b->n + 1;
    if (uni != 0xFFFFFFFFu) {
        // one length (a kv.db partition of fixed-size keys): the offsets are
        // a formula, written on the device instead of copied
        k_fill_offsets<<<grid_for(c, count), 256, 0, c->stream>>>(dst, count, b->key_bytes, uni);
    } else {
        HIP_OK(hipMemcpyAsync(dst, h_off + 1, count * 8, hipMemcpyHostToDevice, c->stream));
        k_rebase_offsets<<<grid_for(c, count), 256, 0, c->stream>>>(dst, count, b->key_bytes - o0);
    }
    HIP_OK(hipStreamSynchronize(c->stream));  // the caller may reuse its buffers
    if ((rc = launch_status())) return rc;
    if (b->n == 0) b->uni_len = uni;
    b->uniform = b->uniform && uni != 0xFFFFFFFFu && uni == b->uni_len;
    b->key_bytes += bytes;
    return BSDB_OK;
}

// Runs an add under the context lock; a failure marks the builder failed.
template <class Add>
int builder_add(bsdb_builder *b, uint64_t count, const uint64_t *h_addr, const uint64_t *h_value8,
                const uint8_t *h_vlen, Add &&add) {
    std::lock_guard<std::mutex> gb(b->mu);
    if (b->failed) return b->failed;
    if (b->finished) return BSDB_EINVAL;
    int rc = builder_check_records(b, count, h_addr, h_value8, h_vlen);
    if (rc) return rc;
    if (count == 0) return BSDB_OK;
    bsdb_ctx *c = b->c;
    {
        std::lock_guard<std::mutex> g(c->mu);
        if (hipSetDevice(c->device) != hipSuccess) return b->failed = BSDB_EIO;
        Ordered ord(c, c->stream);
        rc = add();
    }
    if (!rc) rc = builder_add_records(b, count, h_addr, h_value8, h_vlen);
    if (rc) return b->failed = rc;
    b->n += count;
    return BSDB_OK;
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
    bsdb_mph *p = nullptr;
    auto done = [&](int rc) {
        (void)hipStreamSynchronize(c->stream);
        for (void *q : {d_addr, d_v8, d_vl, slot_a[0], slot_a[1]}) (void)hipFree(q);
        pop_o.finish();
        pop_a.finish();
        if (getenv("BSDB_BUILDER_PROFILE") && fo.map)
            fprintf(stderr, "[bsdb builder] index pages prefaulted in %.3f s (index_a %.3f s)\n", pop_o.seconds, pop_a.seconds);
        if (close_out(fo) && !rc) rc = BSDB_EFILE;
        if (close_out(fao) && !rc) rc = BSDB_EFILE;
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
    pop_o.start(fo.map, fo.bytes, fo.fd, 0);
    pop_a.start(fao.map, fao.bytes, fao.fd, 0);
    fo.pop = &pop_o;
    fao.pop = &pop_a;
    if ((rc = mph_alloc(c, n, width, &p))) return done(rc);
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
        const bool host_gather = getenv("BSDB_BUILDER_HOST_GATHER") != nullptr || rec_bytes > free_b / 4;
        if (!host_gather) {
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
        if (!b->approx && !host_gather) {
            // the solve stores the final slots (addr[p] or base + stride p)
            sink.job = [&](int, const uint64_t *d_slice, uint64_t nl, uint64_t e_lo) {
                return write_slots(c->device, fo, d_slice, nl, e_lo, nullptr, nullptr);
            };
        } else if (!host_gather) {
            // approximate: positions in the slots, gathered on the device
            sink.positions = true;
            sink.job_bytes_per_key = 16;
            sink.prepare = [&](int sl, uint64_t nl) { return grow(&slot_a[sl], &slot_a_bytes[sl], std::max<uint64_t>(nl, 1) * 8); };
            sink.job = [&](int sl, const uint64_t *d_slice, uint64_t nl, uint64_t e_lo) {
                hipStream_t st = nullptr;
                if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return BSDB_EIO;
                k_slot_gather<<<grid_for(c, nl), 256, 0, st>>>(const_cast<uint64_t *>(d_slice), nl, dev_addr,
                                                                b->addr_base, b->addr_stride, (const uint64_t *)d_v8,
                                                                (const uint8_t *)d_vl, (uint64_t *)slot_a[sl]);
                const bool ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
                (void)hipStreamDestroy(st);
                if (!ok) return BSDB_EIO;
                int r = write_slots(c->device, fo, d_slice, nl, e_lo, nullptr, nullptr);
                if (!r) r = write_slots(c->device, fao, (const uint64_t *)slot_a[sl], nl, e_lo, nullptr, nullptr);
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
    rc = passes_build(c, src, n, width, passes, dev_addr, b->addr_base, b->addr_stride, p->E, p->values, p->sigbits,
                      sink, passes_used, c->stream);
    return done(rc);
#undef FIN_OK
}

void builder_release(bsdb_builder *b) {
    b->stop_prefault();
    (void)hipSetDevice(b->c->device);
    (void)hipFree(b->d_keys);
    (void)hipFree(b->d_off);
    b->d_keys = nullptr;
    b->d_off = nullptr;
    b->keys_cap = b->off_cap = 0;
    b->addr.release();
    b->value8.release();
    b->vlen.release();
}

int builder_open(bsdb_ctx *c, uint32_t key_len, uint64_t key_capacity, uint64_t blob_capacity, int approximate,
                 uint64_t addr_base, uint64_t addr_stride, bsdb_builder **out) {
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
    int rc = BSDB_OK;
    {
        std::lock_guard<std::mutex> g(c->mu);
        if (hipSetDevice(c->device) != hipSuccess) {
            rc = BSDB_EIO;
        } else {
            Ordered ord(c, c->stream);
            const uint64_t kb = key_len ? key_capacity * key_len : blob_capacity;
            rc = dev_reserve(c, (void **)&b->d_keys, &b->keys_cap, 0, kb + 16);
            if (!rc && !key_len) {
                rc = dev_reserve(c, (void **)&b->d_off, &b->off_cap, 0, (key_capacity + 1) * 8);
                if (!rc && hipMemsetAsync(b->d_off, 0, 8, c->stream) != hipSuccess) rc = BSDB_EIO;
                if (!rc && hipStreamSynchronize(c->stream) != hipSuccess) rc = BSDB_EIO;
            }
        }
    }
    if (!rc && ((!b->stride && !b->addr.reserve(key_capacity)) ||
                (b->approx && (!b->value8.reserve(key_capacity) || !b->vlen.reserve(key_capacity)))))
        rc = BSDB_ENOMEM;
    if (rc) {
        builder_release(b);
        delete b;
        return rc;
    }
    if (!b->stride && b->addr.cap) b->pop_addr.start(reinterpret_cast<uint8_t *>(b->addr.p), b->addr.cap * 8);
    if (b->approx && b->value8.cap) b->pop_v8.start(reinterpret_cast<uint8_t *>(b->value8.p), b->value8.cap * 8);
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
    int rc = builder_open(c, var ? 0 : key_len, n, blob, approximate, addr_base, h_addr ? 0 : addr_stride, &b);
    if (rc) return rc;
    // the caller's record arrays outlive the call: borrowed, not copied
    b->stop_prefault();
    b->borrowed_records = true;
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
            if (!rc)
                rc = builder_add(b, k1 - k0, nullptr, nullptr, nullptr,
                                 [&] { return builder_add_var_locked(b, h_blob, h_off + k0, k1 - k0, uni); });
        } else {
            k1 = std::min(n, k0 + std::max<uint64_t>(1, BATCH / key_len));
            rc = builder_add(b, k1 - k0, nullptr, nullptr, nullptr,
                             [&] { return builder_add_fixed_locked(b, h_keys + k0 * key_len, key_len, k1 - k0); });
        }
        k0 = k1;
    }
    if (!rc) {
        std::lock_guard<std::mutex> g(c->mu);
        if (hipSetDevice(c->device) != hipSuccess) {
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
    return builder_add(b, count, h_addr, h_value8, h_vlen,
                       [&] { return builder_add_fixed_locked(b, h_keys, key_len, count); });
}

int bsdb_builder_add_var(bsdb_builder *b, const uint8_t *h_blob, const uint64_t *h_off, uint64_t count,
                         const uint64_t *h_addr, const uint64_t *h_value8, const uint8_t *h_vlen) {
    if (!b || b->key_len || (count && (!h_blob || !h_off))) return BSDB_EINVAL;
    uint32_t uni = 0;
    if (count && var_batch_lengths(h_off, count, &uni)) return BSDB_EINVAL;
    return builder_add(b, count, h_addr, h_value8, h_vlen,
                       [&] { return builder_add_var_locked(b, h_blob, h_off, count, uni); });
}

int bsdb_builder_count(const bsdb_builder *b, uint64_t *n) {
    if (!b || !n) return BSDB_EINVAL;
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
        std::lock_guard<std::mutex> g(c->mu);
        HIP_OK(hipSetDevice(c->device));
        Ordered ord(c, c->stream);
        rc = builder_finish_locked(b, width, passes, index_path, index_a_path, out, passes_used);
        b->finished = true;
        builder_release(b);  // the keys leave HBM: the MPHF stays
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

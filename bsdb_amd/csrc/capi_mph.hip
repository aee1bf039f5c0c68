// capi_mph.hip -- host-buffer full build (A5-A11 from host keys), the MPHF
// object (A14 fields / A15 raw dump), batched lookup (F4) and the index
// writer of BSDBWriter.buildIndex (A13, F2/F3).  Included by bsdb_capi.hip.
//   W   = src/main/java/tech/bsdb/write/BSDBWriter.java
//   GOV = src/main/java/it/unimi/dsi/sux4j/mph/GOVMinimalPerfectHashFunctionModified.java

struct bsdb_index;

struct bsdb_mph {
    bsdb_ctx *c = nullptr;  // nullptr once its context was closed (arrays released then)
    int device = 0;
    std::vector<bsdb_index *> ixs;  // its open index writers (detached when it is freed)
    uint64_t n = 0, m = 0;
    uint32_t width = 0;
    uint64_t values_words = 0, sig_words = 0;
    uint64_t *E = nullptr, *values = nullptr, *sigbits = nullptr;  // device
};

struct bsdb_index {
    bsdb_mph *mph = nullptr;  // nullptr once the MPHF was freed
    int device = 0;
    bool approx = false;
    uint64_t pass_size = 0, passes = 0, next_pass = 0, cur = UINT64_MAX;
    FILE *f = nullptr, *fa = nullptr;
    uint64_t *d_index = nullptr;  // the pass's slots (big-endian addresses)
    uint8_t *d_index_a = nullptr; // approximate mode: the pass's 8-byte value slots
};

// Guards the links mph -> context, mph -> index writers and index -> mph:
// bsdb_close / bsdb_mph_free may run (on a garbage collector's thread) before
// the objects that point at them are freed; taken before a context's mph_mu.
static std::mutex g_life_mu;

namespace {

uint64_t mph_sig_words(uint64_t n, uint32_t width) { return width ? (n * width + 63) / 64 + 1 : 0; }

void mph_free_arrays(bsdb_mph *p) {
    (void)hipSetDevice(p->device);
    (void)hipFree(p->E);
    (void)hipFree(p->values);
    (void)hipFree(p->sigbits);
    p->E = p->values = p->sigbits = nullptr;
}

void mph_release(bsdb_mph *p) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> lg(g_life_mu);
        if (p->c) {
            std::lock_guard<std::mutex> g(p->c->mph_mu);
            auto &v = p->c->mphs;
            v.erase(std::remove(v.begin(), v.end(), p), v.end());
        }
        for (bsdb_index *ix : p->ixs) ix->mph = nullptr;  // their later calls return EINVAL
        p->ixs.clear();
    }
    mph_free_arrays(p);
    delete p;
}

// The context an index writer works on, or nullptr when its MPHF was freed or
// the MPHF's context was closed.
bsdb_ctx *index_ctx(const bsdb_index *ix) {
    std::lock_guard<std::mutex> lg(g_life_mu);
    return ix->mph ? ix->mph->c : nullptr;
}

// A new mph on ctx's device with its arrays allocated (not initialised).
int mph_alloc(bsdb_ctx *c, uint64_t n, uint32_t width, bsdb_mph **out) {
    bsdb_mph *p = new (std::nothrow) bsdb_mph();
    if (!p) return BSDB_ENOMEM;
    p->c = c;
    p->device = c->device;
    {
        std::lock_guard<std::mutex> g(c->mph_mu);
        c->mphs.push_back(p);
    }
    p->n = n;
    p->m = n / BUCKET_SIZE + 1;
    p->width = width;
    p->values_words = bsdb_values_words(n);
    p->sig_words = mph_sig_words(n, width);
    if (dmalloc(&p->E, (p->m + 1) * 8) != hipSuccess || dmalloc(&p->values, p->values_words * 8) != hipSuccess ||
        (width && dmalloc(&p->sigbits, p->sig_words * 8) != hipSuccess)) {
        mph_release(p);
        return BSDB_ENOMEM;
    }
    *out = p;
    return BSDB_OK;
}

// hash (host keys -> device signatures) + GOV build into a new mph; with
// d_rank the solve also stores every key's rank by input position (F2).
// The caller holds c->mu and has set the device.
template <class HashDev>
int mph_build_locked(bsdb_ctx *c, uint64_t n, uint32_t width, bsdb_mph **out, int64_t *d_rank, HashDev &&hash_dev) {
    bsdb_mph *p = nullptr;
    int rc = mph_alloc(c, n, width, &p);
    if (rc) return rc;
    void *sig = nullptr;
    if (dmalloc(&sig, std::max<uint64_t>(n, 1) * 16) != hipSuccess) {
        mph_release(p);
        return BSDB_ENOMEM;
    }
    std::unique_ptr<void, DevFree> sig_guard(sig);
    if ((rc = hash_dev((uint64_t *)sig)) ||
        (rc = gov_build_impl(c, (const uint64_t *)sig, n, n, 0, p->m, 0, width, p->E, p->values, p->sigbits, d_rank,
                             c->stream, true))) {
        (void)hipStreamSynchronize(c->stream);
        mph_release(p);
        return rc;
    }
    *out = p;
    return BSDB_OK;
}

template <class HashDev>
int mph_build(bsdb_ctx *c, uint64_t n, uint32_t width, bsdb_mph **out, HashDev &&hash_dev) {
    if (n / BUCKET_SIZE + 1 > 0x7FFFFFFFULL) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    return mph_build_locked(c, n, width, out, nullptr, hash_dev);
}

int write_files(int device, FILE *const *files, const void *const *d_srcs, int nfiles, uint64_t bytes);

// An index file, created/truncated (W:124-127), open for reading too so the
// writer can map it (w+b); a path that cannot be opened so (a write-only
// device) falls back to wb.
FILE *fopen_index(const char *path) {
    FILE *f = fopen(path, "w+b");
    return f ? f : fopen(path, "wb");
}

}  // namespace

// capi_builder.hip: the same files by bucket-range passes (the F2 entry
// points fall back to it when their one-shot build does not fit the device)
static int host_passes_build(bsdb_ctx *c, const uint8_t *h_keys, uint32_t key_len, const uint8_t *h_blob,
                             const uint64_t *h_off, uint64_t n, uint32_t width, const uint64_t *h_addr,
                             uint64_t addr_base, uint64_t addr_stride, const uint64_t *h_value8, const uint8_t *h_vlen,
                             int approximate, uint32_t passes, const char *index_path, const char *index_a_path,
                             bsdb_mph **out, uint32_t *passes_used);
static bool one_shot_fits(bsdb_ctx *c, uint64_t n, bool approx);

namespace {

// F2: build + index.db / index_a.db from the solve's ranks, no rescan.  The
// slots are the same as bsdb_index_* passes over the same records give.
template <class HashDev>
int mph_build_index(bsdb_ctx *c, uint64_t n, uint32_t width, const uint64_t *h_addr, const uint64_t *h_value8,
                    const uint8_t *h_vlen, bool approx, const char *index_path, const char *index_a_path,
                    bsdb_mph **out, HashDev &&hash_dev) {
    if (n / BUCKET_SIZE + 1 > 0x7FFFFFFFULL) return BSDB_EINVAL;
    // W:124-127: both files created first (index_a.db empty in exact mode)
    FILE *f = fopen_index(index_path);
    FILE *fa = index_a_path ? fopen_index(index_a_path) : nullptr;
    auto close_all = [&](int rc) {
        bool ok = true;
        if (f) ok = fclose(f) == 0 && ok;
        if (fa) ok = fclose(fa) == 0 && ok;
        return rc ? rc : (ok ? BSDB_OK : BSDB_EFILE);
    };
    if (!f || (index_a_path && !fa)) return close_all(BSDB_EFILE);
    std::lock_guard<std::mutex> g(c->mu);
    if (hipSetDevice(c->device) != hipSuccess) return close_all(BSDB_EIO);
    Ordered ord(c, c->stream);
    const uint64_t nn = std::max<uint64_t>(n, 1);
    void *rank = nullptr, *addr = nullptr, *index = nullptr, *v8 = nullptr, *vl = nullptr, *index_a = nullptr;
    auto free_all = [&](int rc) {
        (void)hipStreamSynchronize(c->stream);
        for (void *q : {rank, addr, index, v8, vl, index_a}) (void)hipFree(q);
        return close_all(rc);
    };
    if (dmalloc(&rank, nn * 8) != hipSuccess || dmalloc(&addr, nn * 8) != hipSuccess)
        return free_all(BSDB_ENOMEM);
    // the record addresses go up while the MPHF builds (the solve leaves PCIe idle)
    int addr_rc = BSDB_OK;
    std::thread addr_up([&, dev = c->device] { addr_rc = h2d_pageable(dev, addr, h_addr, n * 8); });
    bsdb_mph *p = nullptr;
    int rc = mph_build_locked(c, n, width, &p, (int64_t *)rank, hash_dev);
    addr_up.join();
    if (rc) return free_all(rc);
    if (addr_rc) {
        mph_release(p);
        return free_all(addr_rc);
    }
    if (dmalloc(&index, nn * 8) != hipSuccess ||
        (approx && (dmalloc(&v8, nn * 8) != hipSuccess || dmalloc(&vl, nn) != hipSuccess ||
                    dmalloc(&index_a, nn * 8) != hipSuccess))) {
        mph_release(p);
        return free_all(BSDB_ENOMEM);
    }
    auto chk = [](hipError_t e, const char *what, int line) { return e == hipSuccess || (hip_fail(e, what, line), false); };
    bool ok = chk(hipMemsetAsync(index, 0, nn * 8, c->stream), "memset index", __LINE__);
    if (ok && approx)
        ok = chk(hipMemcpyAsync(v8, h_value8, n * 8, hipMemcpyHostToDevice, c->stream), "H2D value8", __LINE__) &&
             chk(hipMemcpyAsync(vl, h_vlen, n, hipMemcpyHostToDevice, c->stream), "H2D vlen", __LINE__) &&
             chk(hipMemsetAsync(index_a, 0, nn * 8, c->stream), "memset index_a", __LINE__);
    if (ok && n) {
        k_index_scatter<<<grid_for(c, n), 256, 0, c->stream>>>((const int64_t *)rank, (const uint64_t *)addr, n, 0, n,
                                                                (uint64_t *)index, (const uint64_t *)v8,
                                                                (const uint8_t *)vl, (uint8_t *)index_a);
        ok = chk(hipGetLastError(), "k_index_scatter", __LINE__);
    }
    ok = ok && chk(hipStreamSynchronize(c->stream), "sync", __LINE__);
    if (ok) {
        FILE *fs[2] = {f, fa};
        const void *ds[2] = {index, index_a};
        rc = write_files(c->device, fs, ds, approx ? 2 : 1, n * 8);
    } else {
        rc = BSDB_EIO;
    }
    if (rc) {
        mph_release(p);
        return free_all(rc);
    }
    rc = free_all(BSDB_OK);
    if (rc) {
        mph_release(p);
        return rc;
    }
    *out = p;
    return BSDB_OK;
}

// getLong of host keys: per batch the signatures (slot buffer 6) and the
// ranks (buffer 7), copied back into h_out on the compute stream.
template <class Upload>
int mph_lookup_host(bsdb_mph *p, uint64_t n, int check, int64_t *h_out, Upload &&upload_and_hash) {
    bsdb_ctx *c = p->c;
    const MphView v{p->E, p->values, p->sigbits, p->n, (uint32_t)(2 * p->m), p->width};
    int rc = upload_and_hash.template run<true>(c, n, [&](FeedSlot &f, uint64_t k0, uint64_t k1, const uint64_t *d_sig) {
        const uint64_t nk = k1 - k0;
        int r2 = grow(&f.buf[7], &f.cap[7], nk * 8);
        if (r2) return r2;
        k_lookup<<<grid_for(c, nk), 256, 0, c->stream>>>(v, d_sig, nk, check, (int64_t *)f.buf[7]);
        HIP_OK(hipMemcpyAsync(h_out + k0, f.buf[7], nk * 8, hipMemcpyDeviceToHost, c->stream));
        return launch_status();
    });
    if (rc) return rc;
    HIP_OK(hipStreamSynchronize(c->stream));
    return BSDB_OK;
}

// Batched host keys -> device signatures in slot buffer 6, then `then`.
struct FixedKeys {
    const uint8_t *keys;
    uint32_t key_len;
    template <bool, class Then>
    int run(bsdb_ctx *c, uint64_t n, Then &&then) const {
        const uint64_t batch = fixed_batch(key_len, 128ULL << 20);
        return feed_batches(
            c, n, [&](uint64_t k0) { return std::min(n, k0 + batch); },
            [&](FeedSlot &f, uint64_t k0, uint64_t k1) { return upload_fixed(c, f, keys, key_len, k0, k1); },
            [&](FeedSlot &f, uint64_t k0, uint64_t k1) {
                const uint64_t nk = k1 - k0;
                int rc = grow(&f.buf[6], &f.cap[6], nk * 16);
                if (rc) return rc;
                if ((rc = hash_impl(c, (const uint8_t *)f.buf[0], nullptr, nk * key_len, key_len, nk, 0,
                                    (uint64_t *)f.buf[6], c->stream)))
                    return rc;
                return then(f, k0, k1, (const uint64_t *)f.buf[6]);
            });
    }
};

struct VarKeys {
    const uint8_t *blob;
    const uint64_t *off;
    template <bool, class Then>
    int run(bsdb_ctx *c, uint64_t n, Then &&then) const {
        return feed_batches(
            c, n, [&](uint64_t k0) { return var_batch_end(off, k0, n); },
            [&](FeedSlot &f, uint64_t k0, uint64_t k1) { return upload_var(c, f, blob, off, k0, k1); },
            [&](FeedSlot &f, uint64_t k0, uint64_t k1) {
                const uint64_t nk = k1 - k0;
                int rc = grow(&f.buf[6], &f.cap[6], nk * 16);
                if (rc) return rc;
                if ((rc = hash_impl(c, (const uint8_t *)f.buf[0], (const uint64_t *)f.buf[1], off[k1] - off[k0], 0, nk, 0,
                                    (uint64_t *)f.buf[6], c->stream)))
                    return rc;
                return then(f, k0, k1, (const uint64_t *)f.buf[6]);
            });
    }
};

// writeLBuffer (W:166-179): the first `bytes` of a device buffer to the file
// in writes of at most 128 MiB
int write_chunks(FILE *f, const void *d_src, uint64_t bytes, hipStream_t s) {
    constexpr uint64_t CHUNK = 128ULL << 20;
    std::vector<uint8_t> host((size_t)std::min(bytes, CHUNK));
    for (uint64_t o = 0; o < bytes; o += CHUNK) {
        const uint64_t k = std::min(CHUNK, bytes - o);
        HIP_OK(hipMemcpyAsync(host.data(), (const uint8_t *)d_src + o, k, hipMemcpyDeviceToHost, s));
        HIP_OK(hipStreamSynchronize(s));
        if (fwrite(host.data(), 1, k, f) != k) return BSDB_EFILE;
    }
    return BSDB_OK;
}

// The same, fast: each file is cut into 32 MiB writes (the reference writes
// at most 128 MiB at a time) that up to 8 threads issue at their offsets
// (pwrite), each thread staging its pieces through two pooled pinned buffers
// of its own (the DMA of its next piece runs while it writes the current one).
// One thread's fwrite stream ran at ~3 GB/s of page-cache copies; the threads
// share the copies.  The device data must be complete (the caller has
// synchronised its stream).
int write_files(int device, FILE *const *files, const void *const *d_srcs, int nfiles, uint64_t bytes) {
    constexpr uint64_t CHUNK = 128ULL << 20;
    if (bytes <= 2 * CHUNK) {  // small: the plain path (no pinned staging)
        hipStream_t s0 = nullptr;
        for (int i = 0; i < nfiles; ++i) {
            const int rc = write_chunks(files[i], d_srcs[i], bytes, s0);
            if (rc) return rc;
        }
        return BSDB_OK;
    }
    const int ncpu = usable_cpus();
    const uint64_t npieces = (bytes + XFER_PIECE - 1) / XFER_PIECE;
    const uint64_t T = std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)8, (uint64_t)ncpu, npieces}));
    for (int fi = 0; fi < nfiles; ++fi) {
        if (fflush(files[fi]) != 0) return BSDB_EFILE;
        const int fd = fileno(files[fi]);
        const off_t base = ftello(files[fi]);
        if (fd < 0 || base < 0) return BSDB_EFILE;
        const uint8_t *src = (const uint8_t *)d_srcs[fi];
        std::atomic<int> rc{BSDB_OK};
        // a regular file is extended to its new end and the range mapped:
        // parallel pwrite()s to one file serialise on its inode lock, stores
        // into a shared mapping do not (capi_builder.hip's OutFile)
        uint8_t *map = nullptr;
        size_t map_len = 0, map_skip = 0;
        off_t map_base = 0;
        Populator pop;
        {
            struct stat st;
            if (!getenv("BSDB_NO_MMAP_WRITE") && fstat(fd, &st) == 0 && S_ISREG(st.st_mode)) {
                const off_t end = base + (off_t)bytes;
                // (mapped only where the blocks can be reserved ahead of the
                // stores: Populator / file_reserve; otherwise pwrite, which
                // reports a full file system instead of raising SIGBUS)
                const int res = file_reserve(fd, (uint64_t)base, std::min<uint64_t>(bytes, 1u << 16));
                if (res < 0) return BSDB_EFILE;
                if (res == 0 && (st.st_size >= end || ftruncate(fd, end) == 0)) {
                    const off_t pg = (off_t)sysconf(_SC_PAGESIZE);
                    const off_t mbase = base / pg * pg;
                    map_skip = (size_t)(base - mbase);
                    map_len = map_skip + (size_t)bytes;
                    map_base = mbase;
                    void *m = mmap(nullptr, map_len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, mbase);
                    if (m != MAP_FAILED) map = (uint8_t *)m;
                }
            }
        }
        auto work = [&](uint64_t t) {
            hipStream_t st = nullptr;
            void *pin[2] = {nullptr, nullptr};
            hipEvent_t done[2] = {nullptr, nullptr};
            bool ok = hipSetDevice(device) == hipSuccess && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
            for (int i = 0; i < 2 && ok; ++i)
                ok = (pin[i] = pinned_pool().take()) != nullptr &&
                     hipEventCreateWithFlags(&done[i], hipEventDisableTiming) == hipSuccess;
            auto len_of = [&](uint64_t j) { return std::min<uint64_t>(XFER_PIECE, bytes - j * XFER_PIECE); };
            auto issue = [&](uint64_t j, int i) {
                return hipMemcpyAsync(pin[i], src + j * XFER_PIECE, len_of(j), hipMemcpyDeviceToHost, st) == hipSuccess &&
                       hipEventRecord(done[i], st) == hipSuccess;
            };
            if (ok && t < npieces) ok = issue(t, 0);
            int k = 0;
            for (uint64_t j = t; ok && j < npieces; j += T, ++k) {
                const int i = k & 1;
                if (j + T < npieces) ok = issue(j + T, i ^ 1);
                ok = ok && hipEventSynchronize(done[i]) == hipSuccess;
                if (!ok) break;
                const uint64_t len = len_of(j);
                if (map) {
                    if (!pop.ensure(map_skip + j * XFER_PIECE, len)) {
                        rc.store(BSDB_EFILE);
                        ok = false;
                        break;
                    }
                    memcpy(map + map_skip + j * XFER_PIECE, pin[i], len);
                    continue;
                }
                uint64_t w = 0;
                while (w < len) {
                    const ssize_t r = pwrite(fd, (const uint8_t *)pin[i] + w, len - w, base + (off_t)(j * XFER_PIECE + w));
                    if (r <= 0) {
                        rc.store(BSDB_EFILE);
                        ok = false;
                        break;
                    }
                    w += (uint64_t)r;
                }
            }
            if (st) ok = hipStreamSynchronize(st) == hipSuccess && ok;
            if (!ok) {
                int expect = BSDB_OK;
                if (rc.compare_exchange_strong(expect, BSDB_EIO)) (void)hip_fail(hipGetLastError(), "write_files piece", __LINE__);
            }
            for (int i = 0; i < 2; ++i) {
                pinned_pool().give(pin[i]);
                if (done[i]) (void)hipEventDestroy(done[i]);
            }
            if (st) (void)hipStreamDestroy(st);
        };
        pop.start(map, map_len, map ? fd : -1, (uint64_t)map_base);
        std::vector<std::thread> th;
        for (uint64_t t = 1; t < T; ++t) th.emplace_back(work, t);
        work(0);
        for (auto &x : th) x.join();
        pop.finish();
        if (map && munmap(map, map_len) != 0 && !rc.load()) rc.store(BSDB_EFILE);
        if (rc.load()) return rc.load();
        if (fseeko(files[fi], base + (off_t)bytes, SEEK_SET) != 0) return BSDB_EFILE;  // the FILE's position after the data
    }
    (void)hipSetDevice(device);
    return BSDB_OK;
}

// A13 per record batch: rank (checked getLong, W:135) -> slot of this pass
template <class Keys>
int index_put(bsdb_index *ix, const Keys &keys, uint64_t count, const uint64_t *h_addr, const uint64_t *h_value8,
              const uint8_t *h_vlen) {
    bsdb_mph *p = ix->mph;
    bsdb_ctx *c = p ? p->c : nullptr;
    if (!c || ix->cur == UINT64_MAX) return BSDB_EINVAL;  // no pass begun / MPHF gone
    const MphView v{p->E, p->values, p->sigbits, p->n, (uint32_t)(2 * p->m), p->width};
    const uint64_t start = ix->cur * ix->pass_size;
    const uint64_t len = std::min(ix->pass_size, p->n - start);
    return keys.template run<true>(c, count, [&](FeedSlot &f, uint64_t k0, uint64_t k1, const uint64_t *d_sig) {
        const uint64_t nk = k1 - k0;
        int rc;
        if ((rc = grow(&f.buf[2], &f.cap[2], nk * 8)) || (rc = grow(&f.buf[7], &f.cap[7], nk * 8))) return rc;
        // the record payloads go on the compute stream (they are not needed
        // before the scatter, and it keeps the slot's buffers in one order)
        HIP_OK(hipMemcpyAsync(f.buf[2], h_addr + k0, nk * 8, hipMemcpyHostToDevice, c->stream));
        if (ix->approx) {
            if ((rc = grow(&f.buf[3], &f.cap[3], nk * 8)) || (rc = grow(&f.buf[4], &f.cap[4], nk))) return rc;
            HIP_OK(hipMemcpyAsync(f.buf[3], h_value8 + k0, nk * 8, hipMemcpyHostToDevice, c->stream));
            HIP_OK(hipMemcpyAsync(f.buf[4], h_vlen + k0, nk, hipMemcpyHostToDevice, c->stream));
        }
        k_lookup<<<grid_for(c, nk), 256, 0, c->stream>>>(v, d_sig, nk, 1, (int64_t *)f.buf[7]);
        k_index_scatter<<<grid_for(c, nk), 256, 0, c->stream>>>(
            (const int64_t *)f.buf[7], (const uint64_t *)f.buf[2], nk, start, len, ix->d_index,
            ix->approx ? (const uint64_t *)f.buf[3] : nullptr, ix->approx ? (const uint8_t *)f.buf[4] : nullptr,
            ix->approx ? ix->d_index_a : nullptr);
        return launch_status();
    });
}

}  // namespace

// bsdb_close: every MPHF still alive loses its device arrays and its context
static void mph_detach_all(bsdb_ctx *c) {
    std::lock_guard<std::mutex> lg(g_life_mu);
    std::lock_guard<std::mutex> g(c->mph_mu);
    for (bsdb_mph *p : c->mphs) {
        mph_free_arrays(p);
        p->c = nullptr;
    }
    c->mphs.clear();
}

extern "C" {

int bsdb_mph_build_fixed(bsdb_ctx *c, const uint8_t *h_keys, uint32_t key_len, uint64_t n, uint32_t width,
                         bsdb_mph **out) {
    if (!c || !out || bad_key_len(key_len) || width > 64 || (n && !h_keys)) return BSDB_EINVAL;
    *out = nullptr;
    return mph_build(c, n, width, out, [&](uint64_t *d_sig) { return host_hash_fixed_dev(c, h_keys, key_len, n, 0, d_sig); });
}

int bsdb_mph_build_var(bsdb_ctx *c, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n, uint32_t width,
                       bsdb_mph **out) {
    if (!c || !out || width > 64 || (n && (!h_blob || !h_off))) return BSDB_EINVAL;
    *out = nullptr;
    return mph_build(c, n, width, out, [&](uint64_t *d_sig) { return host_hash_var_dev(c, h_blob, h_off, n, 0, d_sig); });
}

int bsdb_mph_build_index_fixed(bsdb_ctx *c, const uint8_t *h_keys, uint32_t key_len, uint64_t n, uint32_t width,
                               const uint64_t *h_addr, const uint64_t *h_value8, const uint8_t *h_vlen,
                               int approximate, const char *index_path, const char *index_a_path, bsdb_mph **out) {
    if (!c || !out || !index_path || bad_key_len(key_len) || width > 64 || (approximate && !index_a_path) ||
        (n && (!h_keys || !h_addr || (approximate && (!h_value8 || !h_vlen)))))
        return BSDB_EINVAL;
    *out = nullptr;
    if (!one_shot_fits(c, n, approximate != 0))
        return host_passes_build(c, h_keys, key_len, nullptr, nullptr, n, width, h_addr, 0, 0, h_value8, h_vlen,
                                 approximate, 0, index_path, index_a_path, out, nullptr);
    return mph_build_index(c, n, width, h_addr, h_value8, h_vlen, approximate != 0, index_path, index_a_path, out,
                           [&](uint64_t *d_sig) { return host_hash_fixed_dev(c, h_keys, key_len, n, 0, d_sig); });
}

int bsdb_mph_build_index_var(bsdb_ctx *c, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n, uint32_t width,
                             const uint64_t *h_addr, const uint64_t *h_value8, const uint8_t *h_vlen, int approximate,
                             const char *index_path, const char *index_a_path, bsdb_mph **out) {
    if (!c || !out || !index_path || width > 64 || (approximate && !index_a_path) ||
        (n && (!h_blob || !h_off || !h_addr || (approximate && (!h_value8 || !h_vlen)))))
        return BSDB_EINVAL;
    *out = nullptr;
    if (!one_shot_fits(c, n, approximate != 0))
        return host_passes_build(c, nullptr, 0, h_blob, h_off, n, width, h_addr, 0, 0, h_value8, h_vlen, approximate, 0,
                                 index_path, index_a_path, out, nullptr);
    return mph_build_index(c, n, width, h_addr, h_value8, h_vlen, approximate != 0, index_path, index_a_path, out,
                           [&](uint64_t *d_sig) { return host_hash_var_dev(c, h_blob, h_off, n, 0, d_sig); });
}

int bsdb_mph_sizes(uint64_t n, uint32_t width, uint64_t *num_buckets, uint64_t *values_words, uint64_t *value_bits,
                   uint64_t *sig_words) {
    if (width > 64 || n / BUCKET_SIZE + 1 > 0x7FFFFFFFULL) return BSDB_EINVAL;  // (GOV:348)
    if (num_buckets) *num_buckets = n / BUCKET_SIZE + 1;
    if (values_words) *values_words = bsdb_values_words(n);
    if (value_bits) *value_bits = 2 * (1 + ((n * 281) >> 8));
    if (sig_words) *sig_words = mph_sig_words(n, width);
    return BSDB_OK;
}

int bsdb_mph_info(const bsdb_mph *p, uint64_t *n, uint64_t *m, uint32_t *width, uint64_t *values_words,
                  uint64_t *sig_words) {
    if (!p) return BSDB_EINVAL;
    if (n) *n = p->n;
    if (m) *m = p->m;
    if (width) *width = p->width;
    if (values_words) *values_words = p->values_words;
    if (sig_words) *sig_words = p->sig_words;
    return BSDB_OK;
}

int bsdb_mph_export(bsdb_mph *p, uint64_t *h_E, uint64_t *h_values, uint64_t *h_sigbits) {
    if (p && !p->c) return BSDB_EINVAL;  // its context was closed
    if (!p || !h_E || !h_values || (p->width && !h_sigbits)) return BSDB_EINVAL;
    bsdb_ctx *c = p->c;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    HIP_OK(hipMemcpyAsync(h_E, p->E, (p->m + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipMemcpyAsync(h_values, p->values, p->values_words * 8, hipMemcpyDeviceToHost, c->stream));
    if (p->width) HIP_OK(hipMemcpyAsync(h_sigbits, p->sigbits, p->sig_words * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    return BSDB_OK;
}

int bsdb_mph_import(bsdb_ctx *c, uint64_t n, uint32_t width, const uint64_t *h_E, const uint64_t *h_values,
                    const uint64_t *h_sigbits, bsdb_mph **out) {
    if (!c || !out || !h_E || !h_values || width > 64 || (width && !h_sigbits) || n / BUCKET_SIZE + 1 > 0x7FFFFFFFULL)
        return BSDB_EINVAL;
    *out = nullptr;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    bsdb_mph *p = nullptr;
    int rc = mph_alloc(c, n, width, &p);
    if (rc) return rc;
    if (hipMemcpyAsync(p->E, h_E, (p->m + 1) * 8, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(p->values, h_values, p->values_words * 8, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        (width && hipMemcpyAsync(p->sigbits, h_sigbits, p->sig_words * 8, hipMemcpyHostToDevice, c->stream) != hipSuccess) ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        mph_release(p);
        return BSDB_EIO;
    }
    *out = p;
    return BSDB_OK;
}

// GOV.dump (GOV:592-619), read back by load_mph (mph.c:28-43)
int bsdb_mph_dump(bsdb_mph *p, const char *path) {
    if (p && !p->c) return BSDB_EINVAL;  // its context was closed
    if (!p || !path) return BSDB_EINVAL;
    std::vector<uint64_t> E(p->m + 1), vals(p->values_words);
    bsdb_ctx *c = p->c;
    {
        std::lock_guard<std::mutex> g(c->mu);
        HIP_OK(hipSetDevice(c->device));
        Ordered ord(c, c->stream);
        HIP_OK(hipMemcpyAsync(E.data(), p->E, E.size() * 8, hipMemcpyDeviceToHost, c->stream));
        HIP_OK(hipMemcpyAsync(vals.data(), p->values, vals.size() * 8, hipMemcpyDeviceToHost, c->stream));
        HIP_OK(hipStreamSynchronize(c->stream));
    }
    FILE *f = fopen(path, "wb");
    if (!f) return BSDB_EFILE;
    const uint64_t head[4] = {p->n, 2 * p->m, 0 /* globalSeed, CBHS:209 */, p->m + 1};
    const uint64_t nv = vals.size();
    bool ok = fwrite(head, 8, 4, f) == 4 && fwrite(E.data(), 8, E.size(), f) == E.size() && fwrite(&nv, 8, 1, f) == 1 &&
              fwrite(vals.data(), 8, vals.size(), f) == vals.size();
    ok = (fclose(f) == 0) && ok;
    return ok ? BSDB_OK : BSDB_EFILE;
}

int bsdb_mph_load(bsdb_ctx *c, const char *path, bsdb_mph **out) {
    if (!c || !path || !out) return BSDB_EINVAL;
    *out = nullptr;
    FILE *f = fopen(path, "rb");
    if (!f) return BSDB_EFILE;
    uint64_t head[4];
    std::vector<uint64_t> E, vals;
    bool ok = fread(head, 8, 4, f) == 4;
    const uint64_t n = head[0], m = n / BUCKET_SIZE + 1;
    // the layout is only ours to read if it is a GOV over n keys: multiplier 2m, m+1 offsets
    ok = ok && head[1] == 2 * m && head[2] == 0 && head[3] == m + 1 && m <= 0x7FFFFFFFULL;
    if (ok) {
        E.resize(m + 1);
        ok = fread(E.data(), 8, E.size(), f) == E.size();
    }
    uint64_t nv = 0;
    ok = ok && fread(&nv, 8, 1, f) == 1 && nv >= bsdb_values_words(n) && nv < (1ULL << 40);
    if (ok) {
        vals.resize(nv);
        ok = fread(vals.data(), 8, nv, f) == nv;
    }
    fclose(f);
    if (!ok) return BSDB_EFILE;
    return bsdb_mph_import(c, n, 0, E.data(), vals.data(), nullptr, out);
}

int bsdb_mph_lookup_fixed(bsdb_mph *p, const uint8_t *h_keys, uint32_t key_len, uint64_t n, int check, int64_t *h_out) {
    if (p && !p->c) return BSDB_EINVAL;  // its context was closed
    if (!p || bad_key_len(key_len) || (n && (!h_keys || !h_out))) return BSDB_EINVAL;
    bsdb_ctx *c = p->c;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    return mph_lookup_host(p, n, check, h_out, FixedKeys{h_keys, key_len});
}

int bsdb_mph_lookup_var(bsdb_mph *p, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n, int check,
                        int64_t *h_out) {
    if (p && !p->c) return BSDB_EINVAL;  // its context was closed
    if (!p || (n && (!h_blob || !h_off || !h_out))) return BSDB_EINVAL;
    bsdb_ctx *c = p->c;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    return mph_lookup_host(p, n, check, h_out, VarKeys{h_blob, h_off});
}

int bsdb_mph_free(bsdb_mph *p) {
    if (!p) return BSDB_EINVAL;
    bsdb_ctx *c = nullptr;
    {
        std::lock_guard<std::mutex> lg(g_life_mu);
        c = p->c;
    }
    if (c) {
        std::lock_guard<std::mutex> g(c->mu);
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
    }
    mph_release(p);
    return BSDB_OK;
}

// ---- A13: the index writer ---------------------------------------------------
int bsdb_index_open(bsdb_mph *p, int approximate, uint64_t pass_cache_bytes, const char *index_path,
                    const char *index_a_path, bsdb_index **out, uint64_t *passes) {
    if (p && !p->c) return BSDB_EINVAL;  // its context was closed
    if (!p || !index_path || !out || (approximate && !index_a_path) || (p->n && pass_cache_bytes && pass_cache_bytes < 8))
        return BSDB_EINVAL;
    *out = nullptr;
    bsdb_index *ix = new (std::nothrow) bsdb_index();
    if (!ix) return BSDB_ENOMEM;
    ix->mph = p;
    ix->device = p->device;
    ix->approx = approximate != 0;
    {
        std::lock_guard<std::mutex> lg(g_life_mu);
        p->ixs.push_back(ix);
    }
    if (!pass_cache_bytes) {  // device-sized pass cache: a quarter of free HBM
        size_t free_b = 0, total_b = 0;
        bool got;
        {
            std::lock_guard<std::mutex> g(p->c->mu);
            got = hipSetDevice(p->c->device) == hipSuccess && hipMemGetInfo(&free_b, &total_b) == hipSuccess;
        }
        if (!got) {
            (void)bsdb_index_close(ix);
            return BSDB_EIO;
        }
        pass_cache_bytes = std::max<uint64_t>(8, free_b / 4 / (ix->approx ? 2 : 1));
    }
    // W:112-118: passSize = min(n, passCacheSize / SLOT_SIZE), passes = ceil(n / passSize)
    ix->pass_size = std::min(p->n, pass_cache_bytes / 8);
    ix->passes = ix->pass_size ? (p->n + ix->pass_size - 1) / ix->pass_size : 0;
    // W:124-127: both files are created (truncated), index_a.db even in exact mode
    ix->f = fopen_index(index_path);
    if (index_a_path) ix->fa = fopen_index(index_a_path);
    bool ok = ix->f && (!index_a_path || ix->fa);
    if (ok && ix->pass_size) {
        bool alloc_ok;
        {
            std::lock_guard<std::mutex> g(p->c->mu);
            alloc_ok = hipSetDevice(p->c->device) == hipSuccess &&
                       dmalloc(&ix->d_index, ix->pass_size * 8) == hipSuccess &&
                       (!ix->approx || dmalloc(&ix->d_index_a, ix->pass_size * 8) == hipSuccess);
        }
        // (bsdb_index_close takes the context lock itself: called after the scope)
        if (!alloc_ok) {
            bsdb_index_close(ix);
            return BSDB_ENOMEM;
        }
    }
    if (!ok) {
        bsdb_index_close(ix);
        return BSDB_EFILE;
    }
    if (passes) *passes = ix->passes;
    *out = ix;
    return BSDB_OK;
}

int bsdb_index_begin_pass(bsdb_index *ix, uint64_t pass) {
    // passes are written to the files in order (W:129-150)
    if (!ix || pass != ix->next_pass || pass >= ix->passes || ix->cur != UINT64_MAX) return BSDB_EINVAL;
    bsdb_ctx *c = index_ctx(ix);
    if (!c) return BSDB_EINVAL;  // its MPHF was freed or its context closed
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    HIP_OK(hipMemsetAsync(ix->d_index, 0, ix->pass_size * 8, c->stream));
    if (ix->approx) HIP_OK(hipMemsetAsync(ix->d_index_a, 0, ix->pass_size * 8, c->stream));
    ix->cur = pass;
    return BSDB_OK;
}

int bsdb_index_put_var(bsdb_index *ix, const uint8_t *h_blob, const uint64_t *h_off, uint64_t count,
                       const uint64_t *h_addr, const uint64_t *h_value8, const uint8_t *h_vlen) {
    if (!ix || (count && (!h_blob || !h_off || !h_addr || (ix->approx && (!h_value8 || !h_vlen))))) return BSDB_EINVAL;
    bsdb_ctx *c = index_ctx(ix);
    if (!c) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    int rc = index_put(ix, VarKeys{h_blob, h_off}, count, h_addr, h_value8, h_vlen);
    if (rc) return rc;
    HIP_OK(hipStreamSynchronize(c->stream));  // the caller may reuse its buffers
    return BSDB_OK;
}

int bsdb_index_put_fixed(bsdb_index *ix, const uint8_t *h_keys, uint32_t key_len, uint64_t count,
                         const uint64_t *h_addr, const uint64_t *h_value8, const uint8_t *h_vlen) {
    if (!ix || bad_key_len(key_len) || (count && (!h_keys || !h_addr || (ix->approx && (!h_value8 || !h_vlen)))))
        return BSDB_EINVAL;
    bsdb_ctx *c = index_ctx(ix);
    if (!c) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    int rc = index_put(ix, FixedKeys{h_keys, key_len}, count, h_addr, h_value8, h_vlen);
    if (rc) return rc;
    HIP_OK(hipStreamSynchronize(c->stream));
    return BSDB_OK;
}

int bsdb_index_end_pass(bsdb_index *ix) {
    if (!ix || ix->cur == UINT64_MAX) return BSDB_EINVAL;
    bsdb_ctx *c = index_ctx(ix);
    if (!c) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    Ordered ord(c, c->stream);
    // W:147: the last pass writes only its lastPassSize slots
    const uint64_t start = ix->cur * ix->pass_size, len = std::min(ix->pass_size, ix->mph->n - start);
    HIP_OK(hipStreamSynchronize(c->stream));
    FILE *fs[2] = {ix->f, ix->fa};
    const void *ds[2] = {ix->d_index, ix->d_index_a};
    int rc = write_files(c->device, fs, ds, ix->approx ? 2 : 1, len * 8);
    if (rc) return rc;
    ix->cur = UINT64_MAX;
    ++ix->next_pass;
    return BSDB_OK;
}

int bsdb_index_close(bsdb_index *ix) {
    if (!ix) return BSDB_EINVAL;
    bool ok = true;
    if (ix->f) ok = fclose(ix->f) == 0 && ok;
    if (ix->fa) ok = fclose(ix->fa) == 0 && ok;
    // unlink from its MPHF (if that is still alive), then release the pass
    // buffers on the writer's own device: the context may be gone already
    bsdb_ctx *c = nullptr;
    {
        std::lock_guard<std::mutex> lg(g_life_mu);
        if (ix->mph) {
            auto &v = ix->mph->ixs;
            v.erase(std::remove(v.begin(), v.end(), ix), v.end());
            c = ix->mph->c;
        }
    }
    if (ix->d_index || ix->d_index_a) {
        if (c) {
            std::lock_guard<std::mutex> g(c->mu);
            (void)hipSetDevice(c->device);
            (void)hipStreamSynchronize(c->stream);
        } else {
            (void)hipSetDevice(ix->device);
            (void)hipDeviceSynchronize();
        }
        (void)hipFree(ix->d_index);
        (void)hipFree(ix->d_index_a);
    }
    // every pass written (W:129-150); a short close leaves short files
    const bool complete = ix->next_pass == ix->passes;
    delete ix;
    return ok ? (complete ? BSDB_OK : BSDB_EINVAL) : BSDB_EFILE;
}

}  // extern "C"

// capi_multi.hip -- E4 behind the C ABI: the full build (MPHF fields +
// index.db / index_a.db) over every device of ONE process (bsdb_multi), the
// form a JVM host drives (the reference's builder is one JVM, SURVEY.md §2.1;
// DESIGN.md §6 describes the same protocol over torch.distributed ranks).
// Included by bsdb_capi.hip after capi_mph.hip.
//   W    = src/main/java/tech/bsdb/write/BSDBWriter.java
//   GOV  = src/main/java/it/unimi/dsi/sux4j/mph/GOVMinimalPerfectHashFunctionModified.java
//   CBHS = src/main/java/it/unimi/dsi/sux4j/io/ConcurrentBucketedHashStore.java
//
// Device g owns buckets [g*m/G, (g+1)*m/G): a contiguous sig0 range (the
// bucket is monotone in sig0, CBHS:129-138), and buckets are independent
// (GOV:405-448).
//  A  every device hashes its input-order shard from host memory, groups the
//     signatures by owner (bsdb_dev_partition_owners, payload = the key's
//     shard position) and gathers the records' addr / value8 / vlen into the
//     same order;
//  B  ONE exchange: every (source, owner) block goes device to device
//     (hipMemcpyPeerAsync: xGMI between MI355X peers), 24 B per key (+9 B in
//     approximate mode);
//  C  every owner solves its range into zeroed full-size arrays
//     (bsdb_dev_gov_build_range; the solve returns each key's rank, F2) and
//     scatters its records' addresses into its index slots [e_lo, e_lo + n_g);
//  D  the fields of different ranges are disjoint bits: each device copies
//     its E entries and the words of its vertex / rank ranges to the host
//     arrays (the two boundary words of a range are OR-ed after all devices
//     finished), and writes its index slice at byte 8*e_lo of the files (W:166-179
//     chunking, pwrite at an offset instead of an append).

namespace {

__global__ __launch_bounds__(256) void k_iota64(uint64_t *out, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) out[i] = i;
}

template <class T>
__global__ __launch_bounds__(256) void k_gather(const uint64_t *perm, const T *src, uint64_t n, T *dst) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) dst[i] = src[perm[i]];
}

// Device allocations of one device of the build, freed on that device.
struct DevBufs {
    int device = 0;
    std::vector<void *> ptrs;
    template <class T>
    int alloc(T **p, uint64_t count) {
        // a fresh host thread's current device is 0: allocate on OUR device
        void *q = nullptr;
        if (hipSetDevice(device) != hipSuccess) return BSDB_EIO;
        if (dmalloc(&q, std::max<uint64_t>(count, 1) * sizeof(T)) != hipSuccess) return BSDB_ENOMEM;
        ptrs.push_back(q);
        *p = (T *)q;
        return BSDB_OK;
    }
    void release(void *q) {
        for (auto &x : ptrs)
            if (x == q) {
                (void)hipSetDevice(device);
                (void)hipFree(x);
                x = nullptr;
            }
    }
    ~DevBufs() {
        (void)hipSetDevice(device);
        for (void *q : ptrs)
            if (q) (void)hipFree(q);
    }
};

struct MultiDev {
    DevBufs mem;
    uint64_t lo = 0, hi = 0;                  // input shard [lo, hi)
    uint64_t cnt[OWN_MAXR] = {};              // shard keys per owner
    uint64_t *sig_g = nullptr, *addr_g = nullptr, *v8_g = nullptr;  // grouped by owner
    uint8_t *vl_g = nullptr;
    uint64_t n_recv = 0, e_lo = 0, b_lo = 0, b_hi = 0;  // owner side
    uint64_t *sig_r = nullptr, *addr_r = nullptr, *v8_r = nullptr;
    uint8_t *vl_r = nullptr;
    // host words OR-ed after every device finished: (index, value), values then sigbits
    std::vector<std::pair<uint64_t, uint64_t>> edge_v, edge_s;
};

// words [a, z) of a device array into h + a: the interior straight into the
// host array, the first and last word into `edge` (OR-ed later: a neighbour
// range may hold bits of the same word)
int copy_words(const uint64_t *d, uint64_t a, uint64_t z, uint64_t *h,
               std::vector<std::pair<uint64_t, uint64_t>> &edge, hipStream_t s) {
    if (a >= z) return BSDB_OK;
    uint64_t w[2] = {0, 0};
    HIP_OK(hipMemcpyAsync(&w[0], d + a, 8, hipMemcpyDeviceToHost, s));
    if (z - a > 1) HIP_OK(hipMemcpyAsync(&w[1], d + z - 1, 8, hipMemcpyDeviceToHost, s));
    if (z - a > 2) HIP_OK(hipMemcpyAsync(h + a + 1, d + a + 1, (z - a - 2) * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    edge.emplace_back(a, w[0]);
    if (z - a > 1) edge.emplace_back(z - 1, w[1]);
    return BSDB_OK;
}

// `bytes` of a device buffer at byte `off` of an open file, in writes of at
// most 128 MiB (W:166-179) through two pinned buffers (chunk i+1 comes over
// PCIe while chunk i is written)
int pwrite_slice(int device, int fd, const void *d_src, uint64_t bytes, uint64_t off) {
    constexpr uint64_t CHUNK = 128ULL << 20;
    if (bytes == 0) return BSDB_OK;
    HIP_OK(hipSetDevice(device));
    hipStream_t st = nullptr;
    void *buf[2] = {nullptr, nullptr};
    const uint64_t cb = std::min(CHUNK, bytes);
    int rc = BSDB_OK;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc(&buf[0], cb, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&buf[1], cb, hipHostMallocDefault) != hipSuccess) {
        rc = BSDB_ENOMEM;
    } else {
        const uint8_t *src = (const uint8_t *)d_src;
        const uint64_t nch = (bytes + CHUNK - 1) / CHUNK;
        auto issue = [&](uint64_t c) {
            const uint64_t o = c * CHUNK, k = std::min(CHUNK, bytes - o);
            return hipMemcpyAsync(buf[c & 1], src + o, k, hipMemcpyDeviceToHost, st) == hipSuccess;
        };
        bool ok = issue(0) && hipStreamSynchronize(st) == hipSuccess;
        for (uint64_t c = 0; ok && c < nch; ++c) {
            if (c + 1 < nch) ok = issue(c + 1);
            const uint64_t k = std::min(CHUNK, bytes - c * CHUNK);
            uint64_t done = 0;
            while (ok && done < k) {
                const ssize_t w = pwrite(fd, (const uint8_t *)buf[c & 1] + done, k - done, (off_t)(off + c * CHUNK + done));
                if (w <= 0) {
                    rc = BSDB_EFILE;
                    ok = false;
                } else {
                    done += (uint64_t)w;
                }
            }
            if (hipStreamSynchronize(st) != hipSuccess) ok = false;
        }
        if (!ok && rc == BSDB_OK) rc = BSDB_EIO;
    }
    if (st) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
    }
    for (void *b : buf)
        if (b) (void)hipHostFree(b);
    return rc;
}

// Runs fn(i) on one host thread per device; the first failure code.
template <class Fn>
int per_device(int k, Fn &&fn) {
    std::vector<int> rcs(k, BSDB_OK);
    std::vector<std::thread> th;
    for (int i = 0; i < k; ++i) th.emplace_back([&, i] { rcs[i] = fn(i); });
    for (auto &t : th) t.join();
    for (int rc : rcs)
        if (rc) return rc;
    return BSDB_OK;
}

template <class HashShard>
int multi_build(bsdb_multi *mc, uint64_t n, uint32_t width, const uint64_t *h_addr, const uint64_t *h_value8,
                const uint8_t *h_vlen, bool approx, const char *index_path, const char *index_a_path, uint64_t *h_E,
                uint64_t *h_values, uint64_t *h_sigbits, HashShard &&hash_shard) {
    const int G = (int)mc->ctx.size();
    const uint64_t m = n / BUCKET_SIZE + 1;
    if (m > 0x7FFFFFFFULL || G > OWN_MAXR) return BSDB_EINVAL;
    const bool index = index_path != nullptr;
    const uint64_t values_words = bsdb_values_words(n), sig_words = mph_sig_words(n, width);
    // BSDB_MULTI_PROFILE=1: wall time of each phase to stderr
    const bool prof = getenv("BSDB_MULTI_PROFILE") != nullptr;
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!prof) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[multi-build] %s %.1f ms\n", what, std::chrono::duration<double, std::milli>(now - t_last).count());
        t_last = now;
    };
    std::vector<MultiDev> dv(G);
    for (int i = 0; i < G; ++i) {
        dv[i].mem.device = mc->ctx[i]->device;
        shard_range(n, G, i, dv[i].lo, dv[i].hi);
        dv[i].b_lo = (uint64_t)i * m / G;
        dv[i].b_hi = (uint64_t)(i + 1) * m / G;
    }
    // W:124-127: the files first, at their final size (index_a.db empty in
    // exact mode); every device then writes its slice in place
    int fd = -1, fda = -1;
    auto close_files = [&](int rc) {
        if (fd >= 0 && close(fd) != 0 && !rc) rc = BSDB_EFILE;
        if (fda >= 0 && close(fda) != 0 && !rc) rc = BSDB_EFILE;
        return rc;
    };
    if (index) {
        fd = open(index_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (index_a_path) fda = open(index_a_path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (fd < 0 || (index_a_path && fda < 0) || ftruncate(fd, (off_t)(8 * n)) != 0 ||
            (approx && ftruncate(fda, (off_t)(8 * n)) != 0))
            return close_files(BSDB_EFILE);
    }
    // peers: direct xGMI copies between distinct devices (a device listed
    // twice copies within itself)
    for (int i = 0; i < G; ++i)
        for (int j = 0; j < G; ++j) {
            const int a = mc->ctx[i]->device, b = mc->ctx[j]->device;
            int can = 0;
            if (a != b && hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can) {
                (void)hipSetDevice(a);
                (void)hipDeviceEnablePeerAccess(b, 0);  // "already enabled" is fine
                (void)hipGetLastError();
            }
        }

    lap("files + peers");
    // ---- A: hash the shard, group by owner, gather the records' payloads
    int rc = per_device(G, [&](int i) -> int {
        bsdb_ctx *c = mc->ctx[i];
        MultiDev &d = dv[i];
        const uint64_t nd = d.hi - d.lo;
        uint64_t *sig = nullptr, *perm = nullptr, *perm_g = nullptr;
        int r;
        HIP_OK(hipSetDevice(c->device));
        if ((r = d.mem.alloc(&sig, 2 * nd)) || (r = d.mem.alloc(&d.sig_g, 2 * nd))) return r;
        if (index && ((r = d.mem.alloc(&perm, nd)) || (r = d.mem.alloc(&perm_g, nd)))) return r;
        {
            std::lock_guard<std::mutex> g(c->mu);
            HIP_OK(hipSetDevice(c->device));
            Ordered ord(c, c->stream);
            if ((r = hash_shard(c, d.lo, d.hi, sig))) return r;
            if (index && nd) k_iota64<<<grid_for(c, nd), 256, 0, c->stream>>>(perm, nd);
            if ((r = launch_status())) return r;
        }
        if ((r = bsdb_dev_partition_owners(c, sig, perm, nd, m, G, d.sig_g, perm_g, d.cnt, c->stream))) return r;
        d.mem.release(sig);
        if (!index) return BSDB_OK;
        std::lock_guard<std::mutex> g(c->mu);
        HIP_OK(hipSetDevice(c->device));
        uint64_t *a = nullptr, *v8 = nullptr;
        uint8_t *vl = nullptr;
        if ((r = d.mem.alloc(&a, nd)) || (r = d.mem.alloc(&d.addr_g, nd))) return r;
        if (approx && ((r = d.mem.alloc(&v8, nd)) || (r = d.mem.alloc(&d.v8_g, nd)) || (r = d.mem.alloc(&vl, nd)) ||
                       (r = d.mem.alloc(&d.vl_g, nd))))
            return r;
        HIP_OK(hipMemcpyAsync(a, h_addr + d.lo, nd * 8, hipMemcpyHostToDevice, c->stream));
        if (approx) {
            HIP_OK(hipMemcpyAsync(v8, h_value8 + d.lo, nd * 8, hipMemcpyHostToDevice, c->stream));
            HIP_OK(hipMemcpyAsync(vl, h_vlen + d.lo, nd, hipMemcpyHostToDevice, c->stream));
        }
        if (nd) {
            k_gather<<<grid_for(c, nd), 256, 0, c->stream>>>(perm_g, a, nd, d.addr_g);
            if (approx) {
                k_gather<<<grid_for(c, nd), 256, 0, c->stream>>>(perm_g, v8, nd, d.v8_g);
                k_gather<<<grid_for(c, nd), 256, 0, c->stream>>>(perm_g, vl, nd, d.vl_g);
            }
        }
        if ((r = launch_status())) return r;
        HIP_OK(hipStreamSynchronize(c->stream));
        for (void *q : {(void *)perm, (void *)perm_g, (void *)a, (void *)v8, (void *)vl}) d.mem.release(q);
        return BSDB_OK;
    });
    if (rc) return close_files(rc);
    lap("A hash + partition + gather");

    // ---- B: the one exchange, every (source, owner) block device to device
    uint64_t acc = 0;
    for (int g = 0; g < G; ++g) {
        dv[g].e_lo = acc;
        for (int i = 0; i < G; ++i) dv[g].n_recv += dv[i].cnt[g];
        acc += dv[g].n_recv;
    }
    if (acc != n) return close_files(BSDB_EIO);
    for (int g = 0; g < G && !rc; ++g) {
        MultiDev &d = dv[g];
        bsdb_ctx *c = mc->ctx[g];
        if (hipSetDevice(c->device) != hipSuccess) { rc = BSDB_EIO; break; }
        if ((rc = d.mem.alloc(&d.sig_r, 2 * d.n_recv))) break;
        if (index && ((rc = d.mem.alloc(&d.addr_r, d.n_recv)))) break;
        if (index && approx && ((rc = d.mem.alloc(&d.v8_r, d.n_recv)) || (rc = d.mem.alloc(&d.vl_r, d.n_recv)))) break;
        uint64_t dst = 0;
        for (int i = 0; i < G && !rc; ++i) {
            const MultiDev &s = dv[i];
            uint64_t src = 0;  // this owner's block in source i's grouped order
            for (int g2 = 0; g2 < g; ++g2) src += s.cnt[g2];
            const uint64_t k = s.cnt[g];
            const int sd = mc->ctx[i]->device, dd = c->device;
            if (k) {
                bool ok = hipMemcpyPeerAsync(d.sig_r + 2 * dst, dd, s.sig_g + 2 * src, sd, k * 16, c->stream) == hipSuccess;
                if (ok && index)
                    ok = hipMemcpyPeerAsync(d.addr_r + dst, dd, s.addr_g + src, sd, k * 8, c->stream) == hipSuccess;
                if (ok && index && approx)
                    ok = hipMemcpyPeerAsync(d.v8_r + dst, dd, s.v8_g + src, sd, k * 8, c->stream) == hipSuccess &&
                         hipMemcpyPeerAsync(d.vl_r + dst, dd, s.vl_g + src, sd, k, c->stream) == hipSuccess;
                if (!ok) rc = BSDB_EIO;
            }
            dst += k;
        }
    }
    for (int g = 0; g < G; ++g) {
        (void)hipSetDevice(mc->ctx[g]->device);
        if (hipStreamSynchronize(mc->ctx[g]->stream) != hipSuccess && !rc) rc = BSDB_EIO;
    }
    if (rc) return close_files(rc);
    for (int i = 0; i < G; ++i)
        for (void *q : {(void *)dv[i].sig_g, (void *)dv[i].addr_g, (void *)dv[i].v8_g, (void *)dv[i].vl_g})
            dv[i].mem.release(q);

    lap("B exchange");
    // ---- C + D: solve each range, copy its fields out, write its index slice
    rc = per_device(G, [&](int g) -> int {
        bsdb_ctx *c = mc->ctx[g];
        MultiDev &d = dv[g];
        if (d.b_lo >= d.b_hi) return d.n_recv ? BSDB_EIO : BSDB_OK;  // more devices than buckets
        HIP_OK(hipSetDevice(c->device));
        uint64_t *E = nullptr, *values = nullptr, *sigbits = nullptr, *idx = nullptr;
        int64_t *rank = nullptr;
        uint8_t *idx_a = nullptr;
        int r;
        if ((r = d.mem.alloc(&E, m + 1)) || (r = d.mem.alloc(&values, values_words)) ||
            (width && (r = d.mem.alloc(&sigbits, sig_words))) || (index && (r = d.mem.alloc(&rank, d.n_recv))))
            return r;
        HIP_OK(hipMemsetAsync(E, 0, (m + 1) * 8, c->stream));
        HIP_OK(hipMemsetAsync(values, 0, values_words * 8, c->stream));
        if (width) HIP_OK(hipMemsetAsync(sigbits, 0, sig_words * 8, c->stream));
        if ((r = bsdb_dev_gov_build_range(c, d.sig_r, d.n_recv, n, d.b_lo, d.b_hi, d.e_lo, width, E, values, sigbits,
                                          rank, c->stream)))
            return r;
        HIP_OK(hipSetDevice(c->device));
        hipStream_t s = c->stream;
        // E[b_lo, b_hi) (+ E[m] on the last range): these entries are this device's alone
        const uint64_t ne = d.b_hi - d.b_lo + (d.b_hi == m ? 1 : 0);
        HIP_OK(hipMemcpyAsync(h_E + d.b_lo, E + d.b_lo, ne * 8, hipMemcpyDeviceToHost, s));
        // the range's vertices [vo(e_lo), vo(e_hi)) (GOV:315-317) hold 2 bits
        // each; the last range also takes the array's tail words
        const uint64_t e_hi = d.e_lo + d.n_recv;
        const uint64_t v_lo = (d.e_lo * 281) >> 8, v_hi = (e_hi * 281) >> 8;
        const bool last = d.b_hi == m;
        if ((r = copy_words(values, (2 * v_lo) / 64, last ? values_words : (2 * v_hi + 63) / 64, h_values, d.edge_v, s)))
            return r;
        if (width && (r = copy_words(sigbits, (d.e_lo * width) / 64, last ? sig_words : (e_hi * width + 63) / 64,
                                     h_sigbits, d.edge_s, s)))
            return r;
        d.mem.release(values);
        d.mem.release(sigbits);
        d.mem.release(E);
        if (!index || d.n_recv == 0) return BSDB_OK;
        if ((r = d.mem.alloc(&idx, d.n_recv)) || (approx && (r = d.mem.alloc(&idx_a, 8 * d.n_recv)))) return r;
        HIP_OK(hipMemsetAsync(idx, 0, d.n_recv * 8, s));
        if (approx) HIP_OK(hipMemsetAsync(idx_a, 0, d.n_recv * 8, s));
        if ((r = bsdb_dev_index_scatter(c, rank, d.addr_r, d.n_recv, d.e_lo, d.n_recv, idx, d.v8_r, d.vl_r, idx_a, s)))
            return r;
        HIP_OK(hipStreamSynchronize(s));
        if ((r = pwrite_slice(c->device, fd, idx, d.n_recv * 8, 8 * d.e_lo))) return r;
        if (approx && (r = pwrite_slice(c->device, fda, idx_a, d.n_recv * 8, 8 * d.e_lo))) return r;
        return BSDB_OK;
    });
    if (rc) return close_files(rc);
    lap("C+D solve + fields + index slices");
    // the boundary words: every contribution OR-ed (fields are disjoint bits)
    auto merge = [&](uint64_t *h, bool sig) {
        for (auto &d : dv)
            for (auto &e : sig ? d.edge_s : d.edge_v) h[e.first] = 0;
        for (auto &d : dv)
            for (auto &e : sig ? d.edge_s : d.edge_v) h[e.first] |= e.second;
    };
    merge(h_values, false);
    if (width) merge(h_sigbits, true);
    return close_files(BSDB_OK);
}

}  // namespace

extern "C" {

int bsdb_multi_mph_build_index_fixed(bsdb_multi *mc, const uint8_t *h_keys, uint32_t key_len, uint64_t n,
                                     uint32_t width, const uint64_t *h_addr, const uint64_t *h_value8,
                                     const uint8_t *h_vlen, int approximate, const char *index_path,
                                     const char *index_a_path, uint64_t *h_E, uint64_t *h_values,
                                     uint64_t *h_sigbits) {
    if (!mc || bad_key_len(key_len) || width > 64 || !h_E || !h_values || (width && !h_sigbits) ||
        (approximate && (!index_path || !index_a_path)) || (n && !h_keys) ||
        (n && index_path && (!h_addr || (approximate && (!h_value8 || !h_vlen)))))
        return BSDB_EINVAL;
    return multi_build(mc, n, width, h_addr, h_value8, h_vlen, approximate != 0, index_path, index_a_path, h_E,
                       h_values, h_sigbits, [&](bsdb_ctx *c, uint64_t lo, uint64_t hi, uint64_t *d_sig) {
                           return host_hash_fixed_dev(c, h_keys + lo * key_len, key_len, hi - lo, 0, d_sig);
                       });
}

int bsdb_multi_mph_build_index_var(bsdb_multi *mc, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n,
                                   uint32_t width, const uint64_t *h_addr, const uint64_t *h_value8,
                                   const uint8_t *h_vlen, int approximate, const char *index_path,
                                   const char *index_a_path, uint64_t *h_E, uint64_t *h_values, uint64_t *h_sigbits) {
    if (!mc || width > 64 || !h_E || !h_values || (width && !h_sigbits) ||
        (approximate && (!index_path || !index_a_path)) || (n && (!h_blob || !h_off)) ||
        (n && index_path && (!h_addr || (approximate && (!h_value8 || !h_vlen)))))
        return BSDB_EINVAL;
    return multi_build(mc, n, width, h_addr, h_value8, h_vlen, approximate != 0, index_path, index_a_path, h_E,
                       h_values, h_sigbits, [&](bsdb_ctx *c, uint64_t lo, uint64_t hi, uint64_t *d_sig) {
                           return host_hash_var_dev(c, h_blob, h_off + lo, hi - lo, 0, d_sig);
                       });
}

}  // extern "C"

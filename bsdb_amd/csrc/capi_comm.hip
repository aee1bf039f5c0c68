// capi_comm.hip -- the histogram stage's one collective
// and the in-process multi-device context, inside the C ABI (B4).  Included by
// bsdb_capi.hip (one translation unit with the kernels).
//
// RCCL is bound at first use with dlopen("librccl.so.1"): in a process that
// already loaded it (torch's) that is the same instance; a Java host gets the
// ROCm one.  Only the stable C entry points below are used; the enum values
// are RCCL's (rccl.h: ncclUint32 = 3, ncclUint64 = 5, ncclSum = 0).

namespace {

typedef int nccl_result_t;
typedef void *nccl_comm_t;
struct nccl_unique_id { char internal[BSDB_COMM_ID_BYTES]; };
constexpr int NCCL_UINT32 = 3, NCCL_UINT64 = 5, NCCL_SUM = 0;

struct Rccl {
    bool tried = false, ok = false;
    nccl_result_t (*get_unique_id)(nccl_unique_id *) = nullptr;
    nccl_result_t (*comm_init_rank)(nccl_comm_t *, int, nccl_unique_id, int) = nullptr;
    nccl_result_t (*comm_init_all)(nccl_comm_t *, int, const int *) = nullptr;
    nccl_result_t (*comm_destroy)(nccl_comm_t) = nullptr;
    nccl_result_t (*all_reduce)(const void *, void *, size_t, int, int, nccl_comm_t, hipStream_t) = nullptr;
    nccl_result_t (*group_start)() = nullptr;
    nccl_result_t (*group_end)() = nullptr;
};

std::mutex g_rccl_mu;
Rccl g_rccl;

const Rccl *rccl() {
    std::lock_guard<std::mutex> g(g_rccl_mu);
    if (g_rccl.tried) return g_rccl.ok ? &g_rccl : nullptr;
    g_rccl.tried = true;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return nullptr;
    Rccl &r = g_rccl;
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
    r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
    r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_init_all && r.comm_destroy && r.all_reduce &&
           r.group_start && r.group_end;
    return r.ok ? &g_rccl : nullptr;
}

// u32 counts -> u16 pairs in one u32 word (low half = even bucket).  A count
// over 65535 is truncated: the sum check after the reduce catches it, since
// every truncation or carry between halves only lowers the unpacked total.
__global__ __launch_bounds__(256) void k_pack16(const uint32_t *counts, uint64_t m, uint32_t *packed) {
    const uint64_t nw = (m + 1) / 2, stride = (uint64_t)gridDim.x * 256;
    for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < nw; w += stride) {
        const uint32_t lo = counts[2 * w] & 0xFFFFu, hi = 2 * w + 1 < m ? counts[2 * w + 1] & 0xFFFFu : 0u;
        packed[w] = lo | (hi << 16);
    }
}

__global__ __launch_bounds__(256) void k_unpack16(const uint32_t *packed, uint64_t m, uint32_t *counts) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < m; b += stride)
        counts[b] = (packed[b >> 1] >> (16 * (b & 1))) & 0xFFFFu;
}

}  // namespace

static void comm_destroy(bsdb_ctx *c) {
    if (c->comm) {
        if (const Rccl *r = rccl()) (void)r->comm_destroy((nccl_comm_t)c->comm);
        c->comm = nullptr;
    }
    c->nranks = 1;
    c->rank = 0;
}

// Sum-all-reduce of the counts and the scan, on the context's communicator.
// counts is an input and receives the global counts.
static int finalize_impl(bsdb_ctx *c, const Rccl *r, uint32_t *d_counts, uint64_t m, uint64_t n_total, uint64_t *d_E,
                         hipStream_t s) {
    int rc;
    const uint64_t nw = (m + 1) / 2;
    if ((rc = grow(&c->pack, &c->pack_bytes, nw * 4))) return rc;
    uint32_t *packed = (uint32_t *)c->pack;
    k_pack16<<<grid_for(c, nw), 256, 0, s>>>(d_counts, m, packed);
    if (r->all_reduce(packed, packed, nw, NCCL_UINT32, NCCL_SUM, (nccl_comm_t)c->comm, s) != 0) return BSDB_ECOMM;
    // unpack into a copy: the u32 retry below needs the local counts intact
    uint32_t *global = (uint32_t *)c->g_counts;
    if ((rc = grow(&c->g_counts, &c->g_counts_bytes, m * 4))) return rc;
    global = (uint32_t *)c->g_counts;
    k_unpack16<<<grid_for(c, m), 256, 0, s>>>(packed, m, global);
    if ((rc = edge_offsets_impl(c, global, m, d_E, s))) return rc;
    uint64_t total = 0;
    HIP_OK(hipMemcpyAsync(&total, d_E + m, 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    if (total != n_total) {
        // a count over 65535 somewhere (every rank sees the same total): u32
        if (r->all_reduce(d_counts, d_counts, m, NCCL_UINT32, NCCL_SUM, (nccl_comm_t)c->comm, s) != 0) return BSDB_ECOMM;
        if ((rc = edge_offsets_impl(c, d_counts, m, d_E, s))) return rc;
        HIP_OK(hipMemcpyAsync(&total, d_E + m, 8, hipMemcpyDeviceToHost, s));
        HIP_OK(hipStreamSynchronize(s));
        return total == n_total ? BSDB_OK : BSDB_ECOMM;
    }
    HIP_OK(hipMemcpyAsync(d_counts, global, m * 4, hipMemcpyDeviceToDevice, s));
    return launch_status();
}

extern "C" {

int bsdb_comm_available(void) { return rccl() ? 1 : 0; }

int bsdb_comm_unique_id(uint8_t *id) {
    if (!id) return BSDB_EINVAL;
    const Rccl *r = rccl();
    if (!r) return BSDB_ECOMM;
    nccl_unique_id u;
    if (r->get_unique_id(&u) != 0) return BSDB_ECOMM;
    memcpy(id, u.internal, BSDB_COMM_ID_BYTES);
    return BSDB_OK;
}

int bsdb_comm_init(bsdb_ctx *c, int nranks, int rank, const uint8_t *id) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return BSDB_EINVAL;
    const Rccl *r = rccl();
    if (!r) return BSDB_ECOMM;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    comm_destroy(c);
    nccl_unique_id u;
    memcpy(u.internal, id, BSDB_COMM_ID_BYTES);
    nccl_comm_t comm = nullptr;
    if (r->comm_init_rank(&comm, nranks, u, rank) != 0) return BSDB_ECOMM;
    c->comm = comm;
    c->nranks = nranks;
    c->rank = rank;
    return BSDB_OK;
}

int bsdb_dev_histogram_finalize(bsdb_ctx *c, uint32_t *d_counts, uint64_t m, uint64_t n_total, uint64_t *d_E,
                                void *stream) {
    if (!c || !d_counts || !d_E || m == 0 || m > 0x7FFFFFFFULL) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->comm) return BSDB_ECOMM;
    const Rccl *r = rccl();
    if (!r) return BSDB_ECOMM;
    HIP_OK(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    Ordered ord(c, s);
    return finalize_impl(c, r, d_counts, m, n_total, d_E, s);
}

int bsdb_dev_allreduce_u64(bsdb_ctx *c, uint64_t *d_buf, uint64_t count, void *stream) {
    if (!c || (count && !d_buf)) return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (!c->comm) return BSDB_ECOMM;
    const Rccl *r = rccl();
    if (!r) return BSDB_ECOMM;
    HIP_OK(hipSetDevice(c->device));
    if (count == 0) return BSDB_OK;
    if (r->all_reduce(d_buf, d_buf, count, NCCL_UINT64, NCCL_SUM, (nccl_comm_t)c->comm, pick(c, stream)) != 0)
        return BSDB_ECOMM;
    return BSDB_OK;
}

}  // extern "C"

// ---- bsdb_multi: every device of this process ----------------------------
struct bsdb_multi {
    std::vector<bsdb_ctx *> ctx;
    std::vector<void *> comms;
    std::vector<uint32_t *> counts;  // per device, m u32 (grown)
    std::vector<uint64_t *> E;       // per device, m+1 u64
    uint64_t m_alloc = 0;
};

namespace {

// shard i of n keys over k devices: contiguous, in input order
inline void shard_range(uint64_t n, int k, int i, uint64_t &lo, uint64_t &hi) {
    lo = n * (uint64_t)i / (uint64_t)k;
    hi = n * (uint64_t)(i + 1) / (uint64_t)k;
}

int multi_grow(bsdb_multi *mc, uint64_t m) {
    if (mc->m_alloc >= m) return BSDB_OK;
    for (size_t i = 0; i < mc->ctx.size(); ++i) {
        HIP_OK(hipSetDevice(mc->ctx[i]->device));
        if (mc->counts[i]) (void)hipFree(mc->counts[i]);
        if (mc->E[i]) (void)hipFree(mc->E[i]);
        mc->counts[i] = nullptr;
        mc->E[i] = nullptr;
        if (dmalloc(&mc->counts[i], m * 4) != hipSuccess || dmalloc(&mc->E[i], (m + 1) * 8) != hipSuccess)
            return BSDB_ENOMEM;
    }
    mc->m_alloc = m;
    return BSDB_OK;
}

// Per device: its shard's histogram from host memory (keys H2D on the
// device's own stream and PCIe link), one host thread per device; then ONE
// grouped all-reduce and the scan on every device; E of device 0 to h_E.
template <class ShardFn>
int multi_histogram(bsdb_multi *mc, uint64_t n, uint64_t *h_E, ShardFn &&shard) {
    const int k = (int)mc->ctx.size();
    const uint64_t m = n / BUCKET_SIZE + 1;
    if (m > 0x7FFFFFFFULL) return BSDB_EINVAL;
    const Rccl *r = rccl();
    if (!r) return BSDB_ECOMM;
    if (!mc->comms[0]) {
        std::vector<int> devs(k);
        for (int i = 0; i < k; ++i) devs[i] = mc->ctx[i]->device;
        if (r->comm_init_all(mc->comms.data(), k, devs.data()) != 0) {
            mc->comms.assign(k, nullptr);
            return BSDB_ECOMM;
        }
    }
    int rc = multi_grow(mc, m);
    if (rc) return rc;
    std::vector<int> rcs(k, BSDB_OK);
    std::vector<std::thread> th;
    for (int i = 0; i < k; ++i)
        th.emplace_back([&, i] {
            bsdb_ctx *c = mc->ctx[i];
            std::lock_guard<std::mutex> g(c->mu);
            if (hipSetDevice(c->device) != hipSuccess) { rcs[i] = BSDB_EIO; return; }
            Ordered ord(c, c->stream);
            if (hipMemsetAsync(mc->counts[i], 0, m * 4, c->stream) != hipSuccess) { rcs[i] = BSDB_EIO; return; }
            rcs[i] = shard(c, i, m, mc->counts[i]);
        });
    for (auto &t : th) t.join();
    for (int i = 0; i < k; ++i)
        if (rcs[i]) return rcs[i];
    // the one collective: the counts summed over xGMI, u16-packed
    for (int i = 0; i < k; ++i) {
        bsdb_ctx *c = mc->ctx[i];
        HIP_OK(hipSetDevice(c->device));
        if ((rc = grow(&c->pack, &c->pack_bytes, ((m + 1) / 2) * 4))) return rc;
        k_pack16<<<grid_for(c, (m + 1) / 2), 256, 0, c->stream>>>(mc->counts[i], m, (uint32_t *)c->pack);
    }
    if (r->group_start() != 0) return BSDB_ECOMM;
    for (int i = 0; i < k; ++i) {
        bsdb_ctx *c = mc->ctx[i];
        (void)hipSetDevice(c->device);
        if (r->all_reduce(c->pack, c->pack, (m + 1) / 2, NCCL_UINT32, NCCL_SUM, (nccl_comm_t)mc->comms[i], c->stream) != 0) {
            (void)r->group_end();
            return BSDB_ECOMM;
        }
    }
    if (r->group_end() != 0) return BSDB_ECOMM;
    bool wide = false;
    for (int pass = 0; pass < 2; ++pass) {
        for (int i = 0; i < k; ++i) {
            bsdb_ctx *c = mc->ctx[i];
            HIP_OK(hipSetDevice(c->device));
            if (!wide) {
                if ((rc = grow(&c->g_counts, &c->g_counts_bytes, m * 4))) return rc;
                k_unpack16<<<grid_for(c, m), 256, 0, c->stream>>>((const uint32_t *)c->pack, m, (uint32_t *)c->g_counts);
                if ((rc = edge_offsets_impl(c, (const uint32_t *)c->g_counts, m, mc->E[i], c->stream))) return rc;
            } else {
                if ((rc = edge_offsets_impl(c, mc->counts[i], m, mc->E[i], c->stream))) return rc;
            }
        }
        uint64_t total = 0;
        HIP_OK(hipSetDevice(mc->ctx[0]->device));
        HIP_OK(hipMemcpyAsync(&total, mc->E[0] + m, 8, hipMemcpyDeviceToHost, mc->ctx[0]->stream));
        for (int i = 0; i < k; ++i) {
            HIP_OK(hipSetDevice(mc->ctx[i]->device));
            HIP_OK(hipStreamSynchronize(mc->ctx[i]->stream));
        }
        if (total == n) break;
        if (wide) return BSDB_ECOMM;
        // a count over 65535: the u32 counts once more
        wide = true;
        if (r->group_start() != 0) return BSDB_ECOMM;
        for (int i = 0; i < k; ++i) {
            (void)hipSetDevice(mc->ctx[i]->device);
            if (r->all_reduce(mc->counts[i], mc->counts[i], m, NCCL_UINT32, NCCL_SUM, (nccl_comm_t)mc->comms[i],
                              mc->ctx[i]->stream) != 0) {
                (void)r->group_end();
                return BSDB_ECOMM;
            }
        }
        if (r->group_end() != 0) return BSDB_ECOMM;
    }
    HIP_OK(hipSetDevice(mc->ctx[0]->device));
    HIP_OK(hipMemcpy(h_E, mc->E[0], (m + 1) * 8, hipMemcpyDeviceToHost));
    return BSDB_OK;
}

}  // namespace

extern "C" {

int bsdb_multi_open(int ndev, const int *devices, bsdb_multi **out) {
    if (!out || ndev < 1 || ndev > 64) return BSDB_EINVAL;
    *out = nullptr;
    bsdb_multi *mc = new (std::nothrow) bsdb_multi();
    if (!mc) return BSDB_ENOMEM;
    std::vector<int> devs(ndev);
    for (int i = 0; i < ndev; ++i) devs[i] = devices ? devices[i] : i;
    mc->ctx.assign(ndev, nullptr);
    mc->comms.assign(ndev, nullptr);
    mc->counts.assign(ndev, nullptr);
    mc->E.assign(ndev, nullptr);
    for (int i = 0; i < ndev; ++i) {
        const int rc = bsdb_open(devs[i], &mc->ctx[i]);
        if (rc) {
            bsdb_multi_close(mc);
            return rc;
        }
    }
    // the RCCL communicator is created by the first call that needs it (the
    // histogram's all-reduce); the full build exchanges device to device
    for (int i = 0; i < ndev; ++i) {
        mc->ctx[i]->nranks = ndev;
        mc->ctx[i]->rank = i;
    }
    *out = mc;
    return BSDB_OK;
}

int bsdb_multi_close(bsdb_multi *mc) {
    if (!mc) return BSDB_EINVAL;
    const Rccl *r = rccl();
    for (size_t i = 0; i < mc->ctx.size(); ++i) {
        if (mc->ctx[i]) (void)hipSetDevice(mc->ctx[i]->device);
        if (mc->comms[i] && r) (void)r->comm_destroy((nccl_comm_t)mc->comms[i]);
        if (mc->counts[i]) (void)hipFree(mc->counts[i]);
        if (mc->E[i]) (void)hipFree(mc->E[i]);
        if (mc->ctx[i]) bsdb_close(mc->ctx[i]);
    }
    delete mc;
    return BSDB_OK;
}

int bsdb_multi_size(const bsdb_multi *mc) { return mc ? (int)mc->ctx.size() : BSDB_EINVAL; }

int bsdb_multi_ctx(bsdb_multi *mc, int i, bsdb_ctx **out) {
    if (!mc || !out || i < 0 || i >= (int)mc->ctx.size()) return BSDB_EINVAL;
    *out = mc->ctx[i];
    return BSDB_OK;
}

int bsdb_multi_histogram_fixed(bsdb_multi *mc, const uint8_t *h_keys, uint32_t key_len, uint64_t n, uint64_t seed,
                               uint64_t *h_E) {
    if (!mc || bad_key_len(key_len) || (n && !h_keys) || !h_E) return BSDB_EINVAL;
    const int k = (int)mc->ctx.size();
    return multi_histogram(mc, n, h_E, [&](bsdb_ctx *c, int i, uint64_t m, uint32_t *d_counts) {
        uint64_t lo, hi;
        shard_range(n, k, i, lo, hi);
        return host_histogram_fixed(c, h_keys + lo * key_len, key_len, hi - lo, seed, m, d_counts);
    });
}

int bsdb_multi_histogram_var(bsdb_multi *mc, const uint8_t *h_blob, const uint64_t *h_off, uint64_t n, uint64_t seed,
                             uint64_t *h_E) {
    if (!mc || (n && (!h_blob || !h_off)) || !h_E) return BSDB_EINVAL;
    const int k = (int)mc->ctx.size();
    return multi_histogram(mc, n, h_E, [&](bsdb_ctx *c, int i, uint64_t m, uint32_t *d_counts) {
        uint64_t lo, hi;
        shard_range(n, k, i, lo, hi);
        return host_histogram_var(c, h_blob, h_off + lo, hi - lo, seed, m, d_counts);
    });
}

}  // extern "C"

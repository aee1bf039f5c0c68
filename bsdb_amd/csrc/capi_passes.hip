// capi_passes.hip -- the full build of a key set resident in ONE device's HBM
// (BASELINE C4: 13 193 787 549 x 13 B = 171.5 GB of keys; C5: 4e9 var-len)
// by sequential bucket-range passes.  Included by bsdb_capi.hip.
//   CBHS = src/main/java/it/unimi/dsi/sux4j/io/ConcurrentBucketedHashStore.java
//   GOV  = src/main/java/it/unimi/dsi/sux4j/mph/GOVMinimalPerfectHashFunctionModified.java
//   W    = src/main/java/tech/bsdb/write/BSDBWriter.java
//
// The reference builds README-size sets in bounded memory: every key's
// signature is spilled to one of 256 segment files by its top byte
// (CBHS:379-395, 497-508), and the segments are read back, sorted and solved
// one at a time (CBHS:852-978 feeding GOV:385-448).  A segment is a contiguous
// sig0 range and so a contiguous bucket range (the bucket is monotone in sig0,
// CBHS:129-138).  Here the keys stay resident and pass p of P covers buckets
// [p*m/P, (p+1)*m/P): every key is re-hashed and the range's keys are
// grouped by bucket with their input position (no spill and no 16-B/key
// signature array: 211 GB at C4), then sorted, solved and signed (A5-A11);
// the solve writes each key's index.db slot itself (A13 with F2: no getLong
// pass).  A pass's slots are contiguous, [E[b_lo], E[b_hi]), and are copied to
// the caller's host array while the next pass runs.

namespace {

// Where a pass's index slots go.  d_index: the device array of all n slots;
// h_index: a host array of all n slots; job: run on a copier thread of its own
// after the pass's solve, with the pass's contiguous slots [e_lo, e_lo + nl)
// in the device buffer d_slice (slot buffer sl = pass & 1, reused two passes
// later), e.g. written to the index files at byte 8 e_lo (the builder,
// capi_builder.hip).  prepare (optional, main thread, before the solve): per
// slot buffer state the job needs for nl slots.  positions: the slots hold
// each key's input position (byte-reversed, as the solve stores addresses)
// for the job to turn into addresses.
struct PassSink {
    uint64_t *d_index = nullptr;
    uint64_t *h_index = nullptr;
    std::function<int(int sl, uint64_t nl)> prepare;
    std::function<int(int sl, const uint64_t *d_slice, uint64_t nl, uint64_t e_lo)> job;
    uint64_t job_bytes_per_key = 0;  // device bytes per key of a pass the job holds (both slot buffers)
    bool positions = false;
    // (optional) where a pass's keys come from when they are not resident:
    // the range's signatures (src.sig, src.n) and each one's add position
    // (*pos: the solve stores it byte-reversed in the key's slot, so the sink
    // works in positions mode); source_bytes_per_key: its device bytes per key
    // of a pass.  The builder's spill mode (capi_builder.hip).
    std::function<int(uint64_t b_lo, uint64_t b_hi, GovSrc &src, const uint64_t **pos)> source;
    uint64_t source_bytes_per_key = 0;
    bool slices() const { return h_index || job; }
};

// device bytes per key of one pass: sorted signature + position payload, plus
// the pass's index slots (twice when they go out of the device: one buffer is
// copied out while the next pass fills the other)
uint64_t pass_bytes_per_key(const PassSink &sink) {
    return 16 + 8 + (sink.slices() ? 16 + sink.job_bytes_per_key : 0) + sink.source_bytes_per_key;
}

int passes_build(bsdb_ctx *c, const GovSrc &src, uint64_t n, uint32_t width, uint32_t passes, const uint64_t *d_addr,
                 uint64_t addr_base, uint64_t addr_stride, uint64_t *d_E, uint64_t *d_values, uint64_t *d_sigbits,
                 const PassSink &sink, uint32_t *passes_used, hipStream_t s) {
    const uint64_t m = n / BUCKET_SIZE + 1;
    // Every bucket's count over the whole set, once, by the histogram stage
    // (binned pass 1 + pass 2: C4 ~43 ms) instead of a re-hash with per-key
    // atomics in every pass (C4: 76 ms x 7).  Its id workspace is sized for
    // 1 G-key chunks and released before the passes are sized.
    GovSrc gsrc = src;
    std::unique_ptr<void, DevFree> counts_all;
    // BSDB_BUILDER_PROFILE=1: per-pass times on stderr
    const bool prof = getenv("BSDB_BUILDER_PROFILE") != nullptr;
    const auto t_start = std::chrono::steady_clock::now();
    auto since = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(); };
    const bool fixed_ok = src.off || (!bad_key_len(src.key_len) && aligned16(src.keys));
    if (n >= (1ULL << 16) && fixed_ok && !sink.source) {
        void *q = nullptr;
        HIP_OK(dmalloc(&q, m * 4));
        counts_all.reset(q);
        HIP_OK(hipMemsetAsync(q, 0, m * 4, s));
        const uint64_t saved_chunk = c->chunk_keys;
        c->chunk_keys = 1ULL << 30;
        const int hrc = histogram_impl(c, src.keys, src.off, src.blob_bytes, src.off ? 0 : src.key_len, n, 0, m,
                                       (uint32_t *)q, s);
        c->chunk_keys = saved_chunk;
        HIP_OK(hipStreamSynchronize(s));
        (void)hipFree(c->ids);
        c->ids = nullptr;
        c->ids_bytes = 0;
        if (hrc) return hrc;
        gsrc.counts_all = (const uint32_t *)q;
    }
    // the per-key buffers of an earlier build on this context are sized for
    // it: released, so the pass count below sees their memory as free (they
    // grow back to this build's pass size)
    HIP_OK(hipStreamSynchronize(s));
    for (void **q : {&c->g_sorted, &c->g_pay}) {
        (void)hipFree(*q);
        *q = nullptr;
    }
    c->g_sorted_bytes = c->g_pay_bytes = 0;
    if (passes == 0) {
        // the fewest passes whose working set fits 85 % of the free HBM (the
        // solver scratch and the per-bucket arrays come on top: ~10 GB)
        size_t free_b = 0, total_b = 0;
        HIP_OK(hipMemGetInfo(&free_b, &total_b));
        const double room = 0.85 * (double)free_b - 12e9;
        const double need = 1.05 * (double)n * (double)pass_bytes_per_key(sink);
        passes = room <= 0 ? 64u : (uint32_t)std::min(64.0, std::max(1.0, std::ceil(need / room)));
    }
    passes = (uint32_t)std::min<uint64_t>(passes, m);
    if (passes_used) *passes_used = passes;
    HIP_OK(hipMemsetAsync(d_values, 0, bsdb_values_words(n) * 8, s));
    if (width) HIP_OK(hipMemsetAsync(d_sigbits, 0, ((n * width + 63) / 64 + 1) * 8, s));
    // two device slice buffers; the copy-out of pass p's slots runs on a
    // thread of its own (own stream) while pass p+1 solves into the other
    void *slice[2] = {nullptr, nullptr};
    size_t slice_bytes[2] = {0, 0};
    std::thread copier[2];
    int copy_rc[2] = {BSDB_OK, BSDB_OK};
    auto join = [&](int i) {
        if (copier[i].joinable()) copier[i].join();
        return copy_rc[i];
    };
    auto finish = [&](int rc) {
        for (int i = 0; i < 2; ++i) {
            const int r = join(i);
            if (!rc) rc = r;
        }
        (void)hipSetDevice(c->device);
        for (void *q : slice) (void)hipFree(q);
        return rc;
    };
    uint64_t e_lo = 0;
    for (uint32_t p = 0; p < passes; ++p) {
        const uint64_t b_lo = (uint64_t)p * m / passes, b_hi = (uint64_t)(p + 1) * m / passes;
        if (b_lo >= b_hi) continue;
        const int sl = (int)(p & 1);
        GovIndexOut ixo;
        ixo.addr = sink.positions ? nullptr : d_addr;
        ixo.addr_base = sink.positions ? 0 : addr_base;
        ixo.addr_stride = sink.positions ? 1 : addr_stride;
        if (sink.d_index) {
            ixo.index = sink.d_index;  // global slots
        } else if (sink.slices()) {
            ixo.idx_lo = e_lo;
            ixo.slots = [&](uint64_t nl) -> uint64_t * {
                if (join(sl)) return nullptr;  // the copy out of this buffer (pass p-2) is done
                if (grow(&slice[sl], &slice_bytes[sl], std::max<uint64_t>(nl, 1) * 8)) return nullptr;
                if (sink.prepare && sink.prepare(sl, nl)) return nullptr;
                return (uint64_t *)slice[sl];
            };
        }  // (neither: the structure only)
        uint64_t nl = 0;
        const double t_pass = since();
        GovSrc psrc = gsrc;
        if (sink.source) {  // the pass's signatures, each with its add position as the slot's "address"
            const uint64_t *pos = nullptr;
            int rs = sink.source(b_lo, b_hi, psrc, &pos);
            if (rs) return finish(rs);
            ixo.addr = pos;
            ixo.addr_base = ixo.addr_stride = 0;
        }
        int rc = gov_build_impl(c, psrc, n, b_lo, b_hi, e_lo, width, d_E, d_values, d_sigbits, nullptr, ixo, s, false, &nl);
        if (rc) return finish(rc);
        if (prof) fprintf(stderr, "[bsdb passes] pass %u: %llu keys, start %.3f s, built in %.3f s\n", p,
                          (unsigned long long)nl, t_pass, since() - t_pass);
        if (sink.slices() && nl) {  // gov_build_impl returned after the device finished
            const uint64_t *src_slots = (const uint64_t *)slice[sl];
            const int dev = c->device;
            const uint64_t lo = e_lo;
            copy_rc[sl] = BSDB_OK;
            if (sink.job) {
                copier[sl] = std::thread([&, src_slots, nl, lo, dev, sl] {
                    (void)hipSetDevice(dev);
                    copy_rc[sl] = sink.job(sl, src_slots, nl, lo);
                });
            } else {
                uint64_t *dst = sink.h_index + e_lo;
                copier[sl] = std::thread([&, dst, src_slots, nl, dev, sl] {
                    copy_rc[sl] = d2h_pageable(dev, dst, src_slots, nl * 8);
                });
            }
        }
        e_lo += nl;
    }
    const double t_join = since();
    const int rc = finish(BSDB_OK);
    if (prof) fprintf(stderr, "[bsdb passes] last slice out %.3f s after the last pass, total %.3f s\n", since() - t_join, since());
    if (rc) return rc;
    return e_lo == n ? BSDB_OK : BSDB_EIO;
}

int passes_entry(bsdb_ctx *c, const GovSrc &src, uint64_t n, uint32_t width, uint32_t passes, const uint64_t *d_addr,
                 uint64_t addr_base, uint64_t addr_stride, uint64_t *d_E, uint64_t *d_values, uint64_t *d_sigbits,
                 uint64_t *d_index, uint64_t *h_index, uint32_t *passes_used, void *stream) {
    const uint64_t m = n / BUCKET_SIZE + 1;
    if (!c || width > 64 || !d_E || !d_values || (width && !d_sigbits) || m > 0x7FFFFFFFULL || passes > 4096 ||
        (d_index && h_index) || (n && !src.keys))
        return BSDB_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OK(hipSetDevice(c->device));
    hipStream_t s = pick(c, stream);
    Ordered ord(c, s);
    PassSink sink;
    sink.d_index = d_index;
    sink.h_index = h_index;
    return passes_build(c, src, n, width, passes, d_addr, addr_base, addr_stride, d_E, d_values, d_sigbits, sink,
                        passes_used, s);
}

}  // namespace

extern "C" {

int bsdb_dev_mph_build_index_passes_fixed(bsdb_ctx *c, const uint8_t *d_keys, uint32_t key_len, uint64_t n,
                                          uint32_t width, uint32_t passes, const uint64_t *d_addr, uint64_t addr_base,
                                          uint64_t addr_stride, uint64_t *d_E, uint64_t *d_values, uint64_t *d_sigbits,
                                          uint64_t *d_index, uint64_t *h_index, uint32_t *passes_used, void *stream) {
    if (bad_key_len(key_len)) return BSDB_EINVAL;
    GovSrc src;
    src.keys = d_keys;
    src.n = n;
    src.key_len = key_len;
    src.blob_bytes = n * key_len;
    return passes_entry(c, src, n, width, passes, d_addr, addr_base, addr_stride, d_E, d_values, d_sigbits, d_index,
                        h_index, passes_used, stream);
}

int bsdb_dev_mph_build_index_passes_var(bsdb_ctx *c, const uint8_t *d_blob, uint64_t blob_bytes, const uint64_t *d_off,
                                        uint64_t n, uint32_t width, uint32_t passes, const uint64_t *d_addr,
                                        uint64_t addr_base, uint64_t addr_stride, uint64_t *d_E, uint64_t *d_values,
                                        uint64_t *d_sigbits, uint64_t *d_index, uint64_t *h_index,
                                        uint32_t *passes_used, void *stream) {
    if (n && !d_off) return BSDB_EINVAL;
    GovSrc src;
    src.keys = d_blob;
    src.off = d_off;
    src.n = n;
    src.blob_bytes = blob_bytes;
    return passes_entry(c, src, n, width, passes, d_addr, addr_base, addr_stride, d_E, d_values, d_sigbits, d_index,
                        h_index, passes_used, stream);
}

}  // extern "C"

// capi_kv.hip -- F3: the kv.db scan that feeds BSDBWriter.buildIndex, native.
// Included by bsdb_capi.hip after capi_mph.hip.  Host code only.
//   W   = src/main/java/tech/bsdb/write/BSDBWriter.java
//   PKV = src/main/java/tech/bsdb/write/PartitionedKVWriter.java
//   SCK = src/main/java/tech/bsdb/write/SimpleCompactKVWriter.java
//   BKV = src/main/java/tech/bsdb/write/BlockedKVWriter.java
//
// buildIndex walks every record of the data files through kvWriter.forEach
// (W:134, PKV:50-70: one task per partition file) and hands each record's
// (address, key, value) to getLong.  The reference allocates two byte[] per
// record (SCK:62-66, BKV:98-103) and re-scans the files once per index pass.
// Here each partition file is mapped and parsed by a host thread into packed
// arrays -- key blob (+ offsets unless every key has one length), record
// address, the first <= 8 value bytes and their count (index_a.db).
// bsdb_kv_scan returns them all (partition order); bsdb_kv_build_index hands
// each partition to the streaming builder as soon as it is parsed (bounded
// host memory; index slots from the solve, no rescan).
//
// Formats (the two uncompressed kv.db layouts):
//   0 compact  SimpleCompactKVWriter: records [kLen u8][vLen u16 BE][key][value]
//              back to back, kLen 0 or end of file ends the partition (SCK:55-70);
//              address = partition << 56 | byte offset (SCK:67).
//   1 blocked  SimpleBlockedKVWriter: blocks of block_size bytes, records never
//              straddle a block, a 0 byte ends a block's records (BKV:67-74);
//              a record longer than a block sits alone in a page-aligned large
//              block (BKV:50-58); address = partition << 56 | block pages << 48
//              | block position in pages << 16 | offset in the block (BKV:124-136).
//              The reference hands a large record's value as null (BKV:105-109,
//              so approximate mode fails there); here its bytes are read.
// The zstd-compressed layout (KVWriterCompressed) is not read: out of scope.

struct bsdb_kv_records {
    uint64_t n = 0;
    uint32_t fixed_len = 0;  // every key this long; 0 when lengths differ (or n == 0)
    std::vector<uint8_t> blob;
    std::vector<uint64_t> off;  // n + 1
    std::vector<uint64_t> addr, value8;
    std::vector<uint8_t> vlen;
};

namespace {

constexpr uint32_t KV_PAGE = 4096;  // NativeFileIO.PAGE_SIZE

// munmap in 32 MiB steps: each munmap holds the address-space lock, which
// another thread's mmap (the finish opening the index file) waits for; a
// partition's ~1 GB released at once held it for tens of ms at a time.
// A releasing thread may be held between steps (the kv.db reaper, while the
// finish allocates: its device allocations waited up to 0.12 s behind it).
thread_local const std::atomic<bool> *t_unmap_hold = nullptr;
void unmap_in_steps(void *p, size_t bytes) {
    constexpr size_t STEP = 32ull << 20;
    for (size_t o = 0; o < bytes; o += STEP) {
        while (t_unmap_hold && t_unmap_hold->load(std::memory_order_acquire))
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        munmap((uint8_t *)p + o, std::min(STEP, bytes - o));
    }
}

// A growable array of plain values, never value-initialised (a partition's
// parse output: written once, record by record).  An anonymous mapping in
// 2 MiB pages where the kernel offers them (MADV_HUGEPAGE): a partition's
// ~400 MB of fresh output otherwise costs ~100 K first-touch page faults on
// its scanning thread.
template <class T>
struct PodBuf {
    T *p = nullptr;
    size_t n = 0, cap = 0;
    PodBuf() = default;
    PodBuf(const PodBuf &) = delete;
    PodBuf &operator=(const PodBuf &) = delete;
    ~PodBuf() { release(); }
    static size_t bytes_of(size_t c) { return (c * sizeof(T) + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1); }
    void reserve(size_t c) {
        if (c <= cap) return;
        const size_t nb = bytes_of(c);
        void *q = p ? mremap(p, bytes_of(cap), nb, MREMAP_MAYMOVE)
                    : mmap(nullptr, nb, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
        if (q == MAP_FAILED) throw std::bad_alloc();
        (void)madvise(q, nb, MADV_HUGEPAGE);
        p = (T *)q;
        cap = nb / sizeof(T);
    }
    T *room(size_t k) {  // space for k more
        if (n + k > cap) reserve(std::max(n + k, cap + cap / 2 + 4096));
        return p + n;
    }
    void release() {
        if (p) unmap_in_steps(p, bytes_of(cap));
        p = nullptr;
        n = cap = 0;
    }
    size_t size() const { return n; }
    T *data() const { return p; }
    T *begin() const { return p; }
    T *end() const { return p + n; }
    T &operator[](size_t i) const { return p[i]; }
};

struct KvPart {
    PodBuf<uint8_t> blob;
    PodBuf<uint64_t> off;  // key offsets into blob, n + 1
    PodBuf<uint64_t> addr, value8;
    PodBuf<uint8_t> vlen;
    bool values = true;  // value8 / vlen wanted (index.approximate, bsdb_kv_scan)
    int rc = BSDB_OK;
    // streamed parse (the kv.db build): every `chunk` records the scanner
    // calls flush(), which adds them to the builder and resets the arrays
    uint64_t chunk = UINT64_MAX;
    std::function<int()> flush;
    void reset_records() {
        blob.n = 0;
        off.n = 1;  // (off[0] == 0: offsets restart with the blob)
        addr.n = 0;
        value8.n = 0;
        vlen.n = 0;
    }
    KvPart() {
        *off.room(1) = 0;
        off.n = 1;
    }
    void reserve(uint64_t records, uint64_t key_bytes) {
        blob.reserve(key_bytes);
        off.reserve(records + 1);
        addr.reserve(records);
        if (values) {
            value8.reserve(records);
            vlen.reserve(records);
        }
    }
    void add(uint64_t a, const uint8_t *key, uint32_t kl, const uint8_t *val, uint32_t vl) {
        memcpy(blob.room(kl), key, kl);
        blob.n += kl;
        off.room(1)[0] = blob.n;
        off.n++;
        addr.room(1)[0] = a;
        addr.n++;
        if (!values) return;
        uint64_t v = 0;
        const uint32_t h = vl < 8 ? vl : 8;
        if (h == 8)
            memcpy(&v, val, 8);  // (little-endian: byte i at bits 8i, W:141)
        else
            for (uint32_t i = 0; i < h; ++i) v |= (uint64_t)val[i] << (8 * i);
        value8.room(1)[0] = v;
        value8.n++;
        vlen.room(1)[0] = (uint8_t)h;
        vlen.n++;
    }
};

struct Mapped {
    const uint8_t *p = nullptr;
    size_t size = 0;
    ~Mapped() {
        if (p && size) unmap_in_steps((void *)p, (size + 4095) & ~(size_t)4095);
    }
    const uint8_t *at(uint64_t pos, uint64_t) const { return p + pos; }  // (the scanners check the bounds)
};

// A kv.db file read through a 4 MiB window (pread) instead of mapped whole:
// the scan parses the same bytes, but no 600 MB file mapping is faulted in
// and torn down per partition.  Those munmaps (page-cache pages, 4 KiB each)
// took 100+ ms a partition under the address-space lock, which the finish's
// device allocations and populators wait for (profiles/r5/kv/).
struct FileWindow {
    static constexpr uint64_t CHUNK = 4ull << 20;
    int fd = -1;
    uint64_t size = 0;
    uint8_t *buf = nullptr;
    uint64_t cap = 0, wb = 0, wl = 0;  // buffer bytes; the window [wb, wb + wl) of the file
    FileWindow() = default;
    FileWindow(const FileWindow &) = delete;
    FileWindow &operator=(const FileWindow &) = delete;
    ~FileWindow() {
        if (fd >= 0) close(fd);
        if (buf) munmap(buf, cap);
    }
    int open_file(const std::string &path) {
        fd = open(path.c_str(), O_RDONLY);
        if (fd < 0) return BSDB_EFILE;
        struct stat st;
        if (fstat(fd, &st) != 0) return BSDB_EFILE;
        size = (uint64_t)st.st_size;
        (void)posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
        return BSDB_OK;
    }
    // the file's bytes [pos, pos + len), or nullptr past its end / on a read error
    const uint8_t *at(uint64_t pos, uint64_t len) {
        if (pos >= wb && pos + len <= wb + wl) return buf + (pos - wb);
        if (pos + len > size) return nullptr;
        const uint64_t want = std::min(std::max(CHUNK, len), size - pos);
        if (want > cap) {
            if (buf) munmap(buf, cap);
            const uint64_t nc = (want + (2ull << 20) - 1) & ~((2ull << 20) - 1);
            void *q = mmap(nullptr, nc, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (q == MAP_FAILED) {
                buf = nullptr;
                cap = wl = 0;
                return nullptr;
            }
            (void)madvise(q, nc, MADV_HUGEPAGE);
            buf = (uint8_t *)q;
            cap = nc;
        }
        uint64_t got = 0;
        while (got < want) {
            const ssize_t r = pread(fd, buf + got, want - got, (off_t)(pos + got));
            if (r < 0 && errno == EINTR) continue;
            if (r <= 0) {
                wl = 0;
                return nullptr;
            }
            got += (uint64_t)r;
        }
        wb = pos;
        wl = got;
        return buf;
    }
};

int map_file(const std::string &path, Mapped &m) {
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) return BSDB_EFILE;
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        return BSDB_EFILE;
    }
    m.size = (size_t)st.st_size;
    if (m.size) {
        void *q = mmap(nullptr, m.size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (q == MAP_FAILED) {
            close(fd);
            m.size = 0;
            return BSDB_EFILE;
        }
        (void)madvise(q, m.size, MADV_SEQUENTIAL);
        m.p = (const uint8_t *)q;
    }
    close(fd);
    return BSDB_OK;
}

// SCK:55-70.  Records starting at or past `limit` are not read (a sample).
// Src: a whole mapping (Mapped) or a read window (FileWindow).
template <class Src>
int scan_compact(Src &m, uint64_t part, KvPart &out, uint64_t limit = UINT64_MAX) {
    uint64_t pos = 0;
    while (pos < m.size && pos < limit) {
        const uint8_t *h = m.at(pos, std::min<uint64_t>(3, m.size - pos));
        if (!h) return BSDB_EFILE;
        const uint32_t kl = h[0];
        if (kl == 0) break;
        if (pos + 3 > m.size) return BSDB_EFILE;
        const uint32_t vl = ((uint32_t)h[1] << 8) | h[2];
        if (pos + 3 + kl + vl > m.size) return BSDB_EFILE;
        const uint8_t *r = m.at(pos, 3 + (uint64_t)kl + vl);
        if (!r) return BSDB_EFILE;
        out.add(part << 56 | pos, r + 3, kl, r + 3 + kl, vl);
        pos += 3 + (uint64_t)kl + vl;
        if (out.addr.n >= out.chunk) {
            const int f = out.flush();
            if (f) return f;
        }
    }
    return BSDB_OK;
}

// BKV:84-121
template <class Src>
int scan_blocked(Src &m, uint64_t part, uint32_t block, KvPart &out, uint64_t limit = UINT64_MAX) {
    uint64_t position = 0;
    while (position < m.size && position < limit) {
        const uint64_t end = std::min<uint64_t>(m.size, position + block);  // readBlockAt: up to one block
        uint64_t next = block;
        uint64_t o = position;
        while (o < end) {
            const uint8_t *h = m.at(o, 1);
            if (!h) return BSDB_EFILE;
            const uint32_t kl = h[0];
            if (kl == 0) break;
            if (o + 3 + kl > end) return BSDB_EFILE;
            if (!(h = m.at(o, 3))) return BSDB_EFILE;
            const uint32_t vl = ((uint32_t)h[1] << 8) | h[2];
            const uint32_t rec_off = (uint32_t)(o - position);
            const uint64_t rec = 3 + (uint64_t)kl + vl;
            if (o + rec <= end) {
                const uint8_t *r = m.at(o, rec);
                if (!r) return BSDB_EFILE;
                out.add(part << 56 | (uint64_t)(block / KV_PAGE) << 48 | (position / KV_PAGE) << 16 | rec_off, r + 3,
                        kl, r + 3 + kl, vl);
                o += rec;
                if (out.addr.n >= out.chunk) {
                    const int f = out.flush();
                    if (f) return f;
                }
            } else {
                // a large record alone in a page-aligned block (BKV:104-109)
                next = (rec + KV_PAGE - 1) / KV_PAGE * KV_PAGE;
                if (position + rec > m.size || o + rec > m.size) return BSDB_EFILE;
                const uint8_t *r = m.at(o, rec);
                if (!r) return BSDB_EFILE;
                out.add(part << 56 | (next / KV_PAGE) << 48 | (position / KV_PAGE) << 16 | rec_off, r + 3, kl,
                        r + 3 + kl, vl);
                if (out.addr.n >= out.chunk) {
                    const int f = out.flush();
                    if (f) return f;
                }
                break;
            }
        }
        position += next;
    }
    return BSDB_OK;
}

// one partition's file, mapped whole (BSDB_KV_READ=window: through the
// read window, measured slower: thread scan 2.3-2.9 s against 1.2-1.7 s for
// C2's 8 partitions, profiles/r5/kv/callH_*)
// (on_size: called with the file's size before the scan, e.g. to reserve)
int scan_file(const std::string &path, int format, uint64_t part, uint32_t block, KvPart &out,
              uint64_t limit = UINT64_MAX, uint64_t *size = nullptr,
              const std::function<void(uint64_t)> &on_size = nullptr, Mapped *keep = nullptr) {
    static const bool use_mmap = !getenv("BSDB_KV_READ") || strcmp(getenv("BSDB_KV_READ"), "window") != 0;
    if (use_mmap) {
        Mapped local;
        Mapped &m = keep ? *keep : local;  // (keep: the caller releases the mapping)
        int rc = map_file(path, m);
        if (size) *size = m.size;
        if (!rc && on_size) on_size(m.size);
        if (!rc) rc = format == 0 ? scan_compact(m, part, out, limit) : scan_blocked(m, part, block, out, limit);
        return rc;
    }
    FileWindow w;
    int rc = w.open_file(path);
    if (size) *size = w.size;
    if (!rc && on_size) on_size(w.size);
    if (!rc) rc = format == 0 ? scan_compact(w, part, out, limit) : scan_blocked(w, part, block, out, limit);
    return rc;
}

}  // namespace

extern "C" {

int bsdb_kv_scan(const char *kv_base, int partitions, int format, uint32_t block_size, int threads,
                 bsdb_kv_records **out) {
    if (!kv_base || !out || partitions < 1 || (format != 0 && format != 1) ||
        (format == 1 && (block_size == 0 || block_size % KV_PAGE)))
        return BSDB_EINVAL;
    *out = nullptr;
    std::vector<KvPart> parts(partitions);
    const int T = std::max(1, std::min(threads > 0 ? threads : usable_cpus(), partitions));
    std::atomic<int> next{0};
    auto worker = [&] {
        for (int p; (p = next.fetch_add(1)) < partitions;) {
            const std::string path = std::string(kv_base) + "." + std::to_string(p);  // PKV:79-81
            parts[p].rc = scan_file(path, format, (uint64_t)p, block_size, parts[p]);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(worker);
    worker();
    for (auto &t : th) t.join();
    for (auto &p : parts)
        if (p.rc) return p.rc;
    bsdb_kv_records *r = new (std::nothrow) bsdb_kv_records();
    if (!r) return BSDB_ENOMEM;
    uint64_t n = 0, bytes = 0;
    for (auto &p : parts) {
        n += p.addr.size();
        bytes += p.blob.size();
    }
    try {
        r->n = n;
        r->blob.reserve(bytes + 16);
        r->off.reserve(n + 1);
        r->addr.reserve(n);
        r->value8.reserve(n);
        r->vlen.reserve(n);
        r->off.push_back(0);
        uint32_t fixed = 0;
        bool same = true;
        for (auto &p : parts) {
            const uint64_t base = r->blob.size();
            for (size_t i = 1; i < p.off.size(); ++i) {
                const uint64_t l = p.off[i] - p.off[i - 1];
                if (!fixed) fixed = (uint32_t)l;
                same = same && l == fixed;
                r->off.push_back(base + p.off[i]);
            }
            r->blob.insert(r->blob.end(), p.blob.begin(), p.blob.end());
            r->addr.insert(r->addr.end(), p.addr.begin(), p.addr.end());
            r->value8.insert(r->value8.end(), p.value8.begin(), p.value8.end());
            r->vlen.insert(r->vlen.end(), p.vlen.begin(), p.vlen.end());
            p.blob.release();  // (peak memory: one partition twice)
        }
        r->fixed_len = n && same ? fixed : 0;
        r->blob.resize(bytes + 16, 0);  // readable slack past the last key
        r->blob.resize(bytes);
    } catch (const std::bad_alloc &) {
        delete r;
        return BSDB_ENOMEM;
    }
    *out = r;
    return BSDB_OK;
}

int bsdb_kv_records_info(const bsdb_kv_records *r, uint64_t *n, uint64_t *key_bytes, uint32_t *fixed_len) {
    if (!r) return BSDB_EINVAL;
    if (n) *n = r->n;
    if (key_bytes) *key_bytes = r->blob.size();
    if (fixed_len) *fixed_len = r->fixed_len;
    return BSDB_OK;
}

int bsdb_kv_records_arrays(const bsdb_kv_records *r, const uint8_t **blob, const uint64_t **off,
                           const uint64_t **addr, const uint64_t **value8, const uint8_t **vlen) {
    if (!r) return BSDB_EINVAL;
    if (blob) *blob = r->blob.data();
    if (off) *off = r->off.data();
    if (addr) *addr = r->addr.data();
    if (value8) *value8 = r->value8.data();
    if (vlen) *vlen = r->vlen.data();
    return BSDB_OK;
}

int bsdb_kv_records_free(bsdb_kv_records *r) {
    if (!r) return BSDB_EINVAL;
    delete r;
    return BSDB_OK;
}

// W:91-155 from the data files, in bounded host memory: the partitions are
// scanned by host threads (one partition per thread at a time) and each one's
// keys go into a builder (capi_builder.hip: keys into HBM, addresses and value
// bytes kept in host memory) as soon as it is parsed, in whatever order the
// threads finish (the files do not depend on it); then the bucket-range-pass
// build writes index.db / index_a.db.  Host memory: the records' addresses
// (+ 9 B per record in approximate mode) and the partitions in flight, not
// every key.  Device capacity (and each partition's host arrays) is reserved
// from the records and key bytes per file byte of a 16 MiB sample of
// partition 0, extrapolated over every file (growth covers the rest).
int bsdb_kv_build_index(bsdb_ctx *c, const char *kv_base, int partitions, int format, uint32_t block_size,
                        int threads, uint32_t width, int approximate, const char *index_path, const char *index_a_path,
                        bsdb_mph **out) {
    if (!c || !out || !index_path || width > 64 || !kv_base || partitions < 1 || (format != 0 && format != 1) ||
        (format == 1 && (block_size == 0 || block_size % KV_PAGE)) || (approximate && !index_a_path))
        return BSDB_EINVAL;
    *out = nullptr;
    // BSDB_BUILDER_PROFILE=1: phase times on stderr
    const bool prof = getenv("BSDB_BUILDER_PROFILE") != nullptr;
    const auto t_start = std::chrono::steady_clock::now();
    auto since = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(); };
    std::atomic<uint64_t> scan_ns{0}, add_ns{0};
    uint64_t file_bytes = 0;
    for (int p = 0; p < partitions; ++p) {
        struct stat st;
        const std::string path = std::string(kv_base) + "." + std::to_string(p);
        if (stat(path.c_str(), &st) != 0) return BSDB_EFILE;
        file_bytes += (uint64_t)st.st_size;
    }
    // records and key bytes per file byte, from the start of EVERY partition
    // (16 MiB in all, at least 64 KiB each): a first partition of shorter keys
    // than the rest no longer under-sizes the device key area (a
    // key area that still cannot grow makes the builder spill, not fail)
    double per_byte_keys = 0.0, per_byte_blob = 0.0;
    {
        const uint64_t each = std::max<uint64_t>(64ull << 10, (16ull << 20) / (uint64_t)partitions);
        uint64_t seen = 0, keys = 0, blob = 0;
        for (int p = 0; p < partitions; ++p) {
            KvPart sample;
            sample.values = false;
            uint64_t size = 0;
            const int rc = scan_file(std::string(kv_base) + "." + std::to_string(p), format, (uint64_t)p, block_size,
                                     sample, each, &size);
            if (rc) return rc;
            seen += std::min<uint64_t>(size, each);
            keys += sample.addr.size();
            blob += sample.blob.size();
        }
        if (seen) {
            per_byte_keys = (double)keys / (double)seen;
            per_byte_blob = (double)blob / (double)seen;
        }
    }
    bsdb_builder *b = nullptr;
    const double t_sampled = since();
    int rc = BSDB_OK;
    std::unique_ptr<bsdb_builder, int (*)(bsdb_builder *)> guard(nullptr, bsdb_builder_free);
    double t_opened = 0;
    // The builder opens on this thread after the scan threads have started:
    // its record arrays' populator holds the address-space lock in steps,
    // and thread stacks created behind it started the scans ~45 ms late.  A
    // scan thread waits for the open only at its first add.
    std::mutex open_mu;
    std::condition_variable open_cv;
    int open_state = 1;  // 1 pending, 0 open, < 0 the open's error
    auto wait_open = [&]() -> int {
        std::unique_lock<std::mutex> g(open_mu);
        open_cv.wait(g, [&] { return open_state != 1; });
        return open_state;
    };
    std::vector<double> tl((size_t)partitions * 4, 0.0);  // per partition: scan start, scan end, add end, handed off
    // records per streamed add (BSDB_KV_CHUNK; 0: the whole partition in one add)
    uint64_t kv_chunk = 1ull << 21;
    if (const char *e = getenv("BSDB_KV_CHUNK")) kv_chunk = strtoull(e, nullptr, 10) ? strtoull(e, nullptr, 10) : UINT64_MAX;
    // A partition's file mapping (~600 MB at C2) and parse arrays (~400 MB)
    // are released by one background thread while
    // the other partitions and the finish run: released by the scanning
    // thread they took 50-180 ms after its add (munmap, serialised by the
    // address-space lock; profiles/r5/kv/kv_release_timeline.err).  Joined
    // before returning.
    struct KvWork {
        Mapped m;  // (the read-window form: none)
        KvPart part;
    };
    std::mutex reap_mu;
    std::condition_variable reap_cv;
    std::deque<std::unique_ptr<KvWork>> reap_q;
    bool reap_end = false;
    std::atomic<bool> reap_hold{false};  // set from the finish's start until its files are open
    std::thread reaper([&] {
        t_unmap_hold = &reap_hold;
        for (;;) {
            std::unique_ptr<KvWork> w;
            {
                std::unique_lock<std::mutex> g(reap_mu);
                reap_cv.wait(g, [&] { return reap_end || !reap_q.empty(); });
                if (reap_q.empty()) return;
                w = std::move(reap_q.front());
                reap_q.pop_front();
            }
            w.reset();
        }
    });
    auto reaper_join = [&] {
        reap_hold.store(false, std::memory_order_release);
        {
            std::lock_guard<std::mutex> g(reap_mu);
            reap_end = true;
        }
        reap_cv.notify_one();
        if (reaper.joinable()) reaper.join();
    };
    struct ReaperGuard {
        std::function<void()> f;
        ~ReaperGuard() { f(); }
    } reaper_guard{reaper_join};
    // (partitions in flight = threads: the host memory bound)
    const int T = std::max(1, std::min(threads > 0 ? threads : usable_cpus(), partitions));
    std::atomic<int> next{0};
    std::atomic<int> err{BSDB_OK};
    auto worker = [&] {
        for (int p; !err.load() && (p = next.fetch_add(1)) < partitions;) {
          {
            const auto t0 = std::chrono::steady_clock::now();
            std::unique_ptr<KvWork> work(new (std::nothrow) KvWork());
            if (!work) {
                int expect = BSDB_OK;
                err.compare_exchange_strong(expect, BSDB_ENOMEM);
                break;
            }
            KvPart &part = work->part;
            part.values = approximate != 0;  // (exact mode: no value bytes)
            // The partition's records go to the builder in chunks as they are
            // parsed (adds from the scan threads run concurrently: the builder
            // reserves each one's ranges under its lock and copies outside
            // it): the copies overlap the other threads' parsing, read a
            // cache-warm chunk, and the parse arrays stay small.
            uint64_t thread_add_ns = 0;
            part.chunk = kv_chunk;
            part.flush = [&]() -> int {
                const uint64_t k = part.addr.size();
                if (!k) return BSDB_OK;
                uint32_t uni = 0;
                int f = var_batch_lengths(part.off.data(), k, &uni);
                if (!f) f = wait_open();
                if (f) return f;
                const auto t1 = std::chrono::steady_clock::now();
                AddBatch a;
                a.keys = part.blob.data();
                a.off = part.off.data();
                a.count = k;
                a.uni = uni;
                f = builder_add(b, a, part.addr.data(), part.value8.data(), part.vlen.data());
                thread_add_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t1).count();
                part.reset_records();
                return f;
            };
            int r;
            try {
                r = scan_file(std::string(kv_base) + "." + std::to_string(p), format, (uint64_t)p, block_size, part,  // PKV:79-81
                              UINT64_MAX, nullptr, [&](uint64_t size) {
                                  const uint64_t recs = (uint64_t)(per_byte_keys * (double)size * 1.05) + 64;
                                  const uint64_t want = kv_chunk == UINT64_MAX ? recs : std::min<uint64_t>(recs, kv_chunk + 64);
                                  part.reserve(want, (uint64_t)(per_byte_blob / std::max(per_byte_keys, 1e-12) *
                                                                (double)want * 1.05) + 4096);
                              }, &work->m);
                tl[4 * (size_t)p + 1] = since();
                if (!r) r = part.flush();  // the rest
            } catch (const std::bad_alloc &) {
                r = BSDB_ENOMEM;
            }
            tl[4 * (size_t)p] = std::chrono::duration<double>(t0 - t_start).count();
            tl[4 * (size_t)p + 2] = since();
            add_ns += thread_add_ns;
            scan_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() - thread_add_ns;
            if (r) {
                int expect = BSDB_OK;
                err.compare_exchange_strong(expect, r);
            }
            {
                std::lock_guard<std::mutex> g(reap_mu);
                reap_q.push_back(std::move(work));  // (released by the reaper)
            }
            reap_cv.notify_one();
          }
          tl[4 * (size_t)p + 3] = since();
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(worker);
    rc = builder_open(c, 0, (uint64_t)(per_byte_keys * (double)file_bytes * 1.02) + 1024,
                      (uint64_t)(per_byte_blob * (double)file_bytes * 1.02) + 65536, approximate, 0, 0, &b);
    guard.reset(rc ? nullptr : b);
    t_opened = since();
    {
        std::lock_guard<std::mutex> g(open_mu);
        open_state = rc ? rc : 0;
    }
    open_cv.notify_all();
    if (!rc) worker();
    for (auto &t : th) t.join();
    if (rc) return rc;
    if ((rc = err.load())) return rc;
    const double t_scanned = since();
    if (prof) {
        fprintf(stderr, "[bsdb kv] sampled %.3f s, builder open %.3f s, %d threads; partitions (scan start, scan end, add end, released):",
                t_sampled, t_opened, T);
        for (int p = 0; p < partitions; ++p)
            fprintf(stderr, " %d:(%.3f %.3f %.3f %.3f)", p, tl[4 * p], tl[4 * p + 1], tl[4 * p + 2], tl[4 * p + 3]);
        fprintf(stderr, "\n");
    }
    reap_hold.store(true, std::memory_order_release);
    // The reaper waits out the whole finish: released beside it, the munmaps
    // delayed its allocations and first pass by 50-150 ms; held, the finish
    // takes 0.25-0.27 s and the release 0.06-0.15 s after it (C2: 148-168 M
    // keys/s against 138-161 M, profiles/r5/kv/callI_*).  BSDB_KV_REAP_HOLD=open
    // (measurement): held only until the finish's files and arrays exist.
    static const bool hold_open = getenv("BSDB_KV_REAP_HOLD") && !strcmp(getenv("BSDB_KV_REAP_HOLD"), "open");
    if (hold_open) b->on_opened = [&] { reap_hold.store(false, std::memory_order_release); };
    rc = bsdb_builder_finish(b, width, 0, index_path, index_a_path, out, nullptr);
    reap_hold.store(false, std::memory_order_release);
    const double t_finished = since();
    reaper_join();
    if (prof)
        fprintf(stderr, "[bsdb kv] %llu records: scan+add %.3f s (thread scan %.3f s, thread adds %.3f s), finish %.3f s, "
                        "partitions released %.3f s after\n",
                (unsigned long long)b->n, t_scanned, scan_ns.load() / 1e9, add_ns.load() / 1e9, t_finished - t_scanned,
                since() - t_finished);
    return rc;
}

}  // extern "C"

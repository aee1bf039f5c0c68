// jni/GpuBSDBWriter.java -- the MI355X drop-in for tech.bsdb.write.BSDBWriter
// (src/main/java/tech/bsdb/write/BSDBWriter.java, "W"): the same public
// constructor and methods (W:39,67,71,75,91,99,107), the same kv.db writers
// and the same output files (kv.db.<p>, config.properties, hash.db, index.db,
// index_a.db), with the key hash, bucket histogram, GOV solve, signing and the
// index scatter on the GPU through GpuBuild (jni/GpuBuild.java, the C ABI of
// include/bsdb_mi355x.h).  The reference's BSDBWriter delegates every public
// method to it when the JVM runs with -Dbsdb.build.gpu=true (jni/BSDBWriter-gpu.patch,
// off by default), so its callers -- Builder.java:86, ParquetBuilder.java:90,
// BSDBWriterTest.java:34 -- construct BSDBWriter unchanged.
//
// What replaces what:
//   put     W:75-89 appends to the KV writer, then keys.add(key) hashes the key
//           into the 24-byte spill of ConcurrentBucketedHashStore (CBHS:360-395).
//           Here the KV writer is the same; for the data layouts the library
//           reads itself (compact, blocked) the key needs nothing more, since
//           build() takes the keys from the finished kv.db files; for the
//           compressed layout each put() thread batches keys in direct buffers
//           that go into a device builder (bsdb_builder_add_var: keys into HBM).
//   build   W:91-97.  Compact / blocked: ONE call, bsdb_kv_build_index (the
//           files scanned on host threads with the reference's record
//           addresses, the keys streamed into HBM, the MPHF built by bucket-range
//           passes, index.db / index_a.db written from the solve's ranks), then
//           hash.db.  Compressed: buildHash() then buildIndex() as the reference.
//   buildHash  W:99-105: the MPHF from the device, turned into the reference's
//           own GOVMinimalPerfectHashFunctionModified (GovAssembler) and stored
//           with the same BinIO.storeObject call, so Reader.java:30 loads it.
//   buildIndex W:107-155: the reference's pass loop (passSize = min(n, ps/8),
//           one kvWriter.forEach per pass) with each record's getLong done in
//           batches on the device (bsdb_index_put_var) and <= 128 MiB writes
//           (W:166-179, bsdb_index_end_pass); nothing to do after the one-call
//           build.
//
// Not compiled here: this image and the GPU box have no JDK (INTEGRATION.md);
// tests/test_jni_shim.py checks that every simple name resolves.
package tech.bsdb.write;

import it.unimi.dsi.fastutil.io.BinIO;
import it.unimi.dsi.sux4j.mph.GOVMinimalPerfectHashFunctionModified;
import org.apache.commons.configuration2.Configuration;
import org.apache.commons.configuration2.PropertiesConfiguration;
import org.apache.commons.configuration2.builder.FileBasedConfigurationBuilder;
import org.apache.commons.configuration2.builder.fluent.Configurations;
import org.apache.commons.configuration2.ex.ConfigurationException;
import sun.nio.ch.DirectBuffer;
import tech.bsdb.gpu.GovAssembler;
import tech.bsdb.gpu.GpuBuild;

import java.io.File;
import java.io.IOException;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayDeque;
import java.util.ArrayList;
import java.util.List;
import java.util.Objects;
import java.util.concurrent.atomic.AtomicLong;

import static tech.bsdb.util.Common.*;

public class GpuBSDBWriter {
    /** HIP device of this writer (-Dbsdb.gpu.device, default 0). */
    private static final int DEVICE = Integer.getInteger("bsdb.gpu.device", 0);
    /** Keys (and key bytes) one put() thread collects before they go to the device. */
    private static final int BATCH_KEYS = 1 << 18, BATCH_BYTES = 16 << 20;

    private final File basePath;
    private final KVWriter kvWriter;
    private final int checksumBits;
    private final long passCacheSize;
    private final boolean approximateMode;
    private final AtomicLong recordCount = new AtomicLong(0);
    private final Configuration config;
    private final FileBasedConfigurationBuilder<PropertiesConfiguration> configBuilder;
    private final long ctx;
    /** kv.db layout the library scans (0 compact, 1 blocked), or -1 (compressed: keys batched from put). */
    private final int nativeFormat;
    private final long builder;
    private final List<Batch> batches = new ArrayList<>();
    private final ThreadLocal<Batch> keyBatch;
    private long gpuMph;
    private boolean indexWritten;

    public GpuBSDBWriter(File basePath, File tmpDir, int checksumBits, long passCacheSize, boolean compact,
                         boolean compress, int compressBlockSize, int sharedDictSize, boolean approximateMode)
            throws Exception {
        this.basePath = basePath;
        final File kvFile = new File(basePath, FILE_NAME_KV_DATA);
        if (compress) kvWriter = new KVWriterCompressed(kvFile, compressBlockSize, sharedDictSize, false);
        else if (compact) kvWriter = new SimpleCompactKVWriter(kvFile);
        else kvWriter = new SimpleBlockedKVWriter(kvFile);
        nativeFormat = compress ? -1 : compact ? 0 : 1;
        this.checksumBits = checksumBits;
        this.passCacheSize = passCacheSize;
        this.approximateMode = approximateMode;
        // (tmpDir: the reference's CBHS spill directory; the keys stay in HBM here)
        final File configFile = new File(basePath, FILE_NAME_CONFIG);
        if (!configFile.exists() && !configFile.createNewFile()) throw new IOException("cannot create " + configFile);
        configBuilder = new Configurations().propertiesBuilder(configFile);
        config = configBuilder.getConfiguration();
        // the same config.properties keys as the reference (Common.java:26-49)
        config.setProperty(CONFIG_KEY_KV_COMPRESS, Boolean.toString(compress));
        config.setProperty(CONFIG_KEY_KV_COMPACT, Boolean.toString(compact));
        config.setProperty(CONFIG_KEY_KV_COMPRESS_BLOCK_SIZE, compressBlockSize);
        config.setProperty(CONFIG_KEY_APPROXIMATE_MODE, Boolean.toString(approximateMode));
        config.setProperty(CONFIG_KEY_CHECKSUM_BITS, checksumBits);
        ctx = GpuBuild.open(DEVICE);
        // the MPHF-only builder of the compressed layout: addresses are not
        // needed at put time (buildIndex rescans the records), so the builder
        // takes the formula form (stride 1) and keeps no record arrays
        builder = nativeFormat < 0 ? GpuBuild.builderOpen(ctx, 0, BATCH_KEYS, BATCH_BYTES, false, 0, 1) : 0;
        keyBatch = ThreadLocal.withInitial(() -> {
            final Batch b = new Batch(false, false);
            synchronized (batches) {
                batches.add(b);
            }
            return b;
        });
    }

    public void sample(byte[] key, byte[] value) {
        kvWriter.sample(key, value);
    }

    public void onSampleFinished() {
        kvWriter.onSampleFinished();
    }

    /** W:75-89; called concurrently (Builder.java:144-160). */
    public void put(byte[] key, byte[] value) throws IOException, InterruptedException {
        if (Objects.isNull(key) || Objects.isNull(value))
            throw new RuntimeException("currently null key/value is not support.");  // W:76-79
        kvWriter.put(key, value);
        if (nativeFormat < 0) {
            final Batch b = keyBatch.get();
            synchronized (b) {
                if (!b.fits(key, null)) b.flushKeys(builder);
                b.add(0, key, null);
            }
        }
        recordCount.getAndIncrement();
    }

    /** W:91-97 */
    public void build() throws IOException, InterruptedException {
        kvWriter.finish();
        kvWriter.getStatistics().writeTo(config);
        try {
            configBuilder.save();
        } catch (ConfigurationException e) {
            throw new RuntimeException(e);
        }
        buildIndex(buildHash());
    }

    /** W:99-105: hash.db stays a serialized GOVMinimalPerfectHashFunctionModified. */
    public GOVMinimalPerfectHashFunctionModified<byte[]> buildHash() throws IOException {
        if (nativeFormat >= 0) {
            // F3: MPHF + index.db / index_a.db from the finished data files in one call
            final PartitionedKVWriter pw = (PartitionedKVWriter) kvWriter;
            final int blockSize = nativeFormat == 1 ? ((BlockedKVWriter) kvWriter).blockSize : 0;
            gpuMph = GpuBuild.kvBuildIndex(ctx, new File(basePath, FILE_NAME_KV_DATA).getPath(), pw.partitions,
                    nativeFormat, blockSize, 0, checksumBits, approximateMode, indexFile().getPath(),
                    approximateIndexFile().getPath());
            indexWritten = true;
        } else {
            synchronized (batches) {
                for (Batch b : batches) {
                    synchronized (b) {
                        b.flushKeys(builder);
                    }
                }
            }
            gpuMph = GpuBuild.builderFinish(builder, checksumBits, 0, null, null);  // the MPHF only
            GpuBuild.builderFree(builder);
        }
        final GOVMinimalPerfectHashFunctionModified<byte[]> f = GovAssembler.fromMph(gpuMph);
        BinIO.storeObject(f, new File(basePath, FILE_NAME_KEY_HASH));
        return f;
    }

    /** W:107-155 (the one-call build already wrote both files). */
    public void buildIndex(GOVMinimalPerfectHashFunctionModified<byte[]> hashFunction)
            throws IOException, InterruptedException {
        try {
            if (!indexWritten) passLoop();
        } finally {
            GpuBuild.mphFree(gpuMph);
            GpuBuild.close(ctx);
        }
    }

    // W:112-155: passSize = min(n, ps/8) slots a pass, one kvWriter.forEach per
    // pass; the records go to the device in batches (getLong + scatter there).
    // kvWriter.forEach starts a new thread pool on every call (Common.java:287),
    // so a batch belongs to a pass: the pass's threads take batches from a pool,
    // and every batch goes back to it after the pass's final flush.  The pool
    // holds at most one pass's worth of scan threads' batches.
    private void passLoop() throws IOException, InterruptedException {
        final long[] passes = new long[1];
        final long ix = GpuBuild.indexOpen(gpuMph, approximateMode, passCacheSize, indexFile().getPath(),
                approximateIndexFile().getPath(), passes);
        final ArrayDeque<Batch> pool = new ArrayDeque<>();
        try {
            for (long p = 0; p < passes[0]; p++) {
                GpuBuild.indexBeginPass(ix, p);
                final List<Batch> inPass = new ArrayList<>();
                final ThreadLocal<Batch> records = ThreadLocal.withInitial(() -> {
                    synchronized (pool) {
                        final Batch b = pool.isEmpty() ? new Batch(true, approximateMode) : pool.pop();
                        inPass.add(b);
                        return b;
                    }
                });
                kvWriter.forEach((addr, key, value) -> {   // scan threads (PartitionedKVWriter.java:50-70)
                    final Batch b = records.get();
                    if (!b.fits(key, value)) b.flushRecords(ix, this);
                    b.add(addr, key, value);
                });
                synchronized (pool) {
                    for (Batch b : inPass) b.flushRecords(ix, this);
                    pool.addAll(inPass);                      // the next pass's threads reuse them
                }
                GpuBuild.indexEndPass(ix);                    // the pass's <= 128 MiB writes (W:166-179)
            }
        } finally {
            GpuBuild.indexClose(ix);
        }
    }

    private File indexFile() {
        return new File(basePath, FILE_NAME_KV_INDEX);
    }

    private File approximateIndexFile() {
        return new File(basePath, FILE_NAME_KV_APPROXIMATE_INDEX);
    }

    /** One thread's keys (and, for the pass loop, records) in direct buffers the C ABI reads in place. */
    private static final class Batch {
        final ByteBuffer blob = direct(BATCH_BYTES);
        final ByteBuffer offs = direct(8L * (BATCH_KEYS + 1));
        final ByteBuffer addr, value8, vlen;
        int count;

        /** records: a pass loop's batch (addresses); approximate: index_a.db value bytes too (W:140-142). */
        Batch(boolean records, boolean approximate) {
            addr = records ? direct(8L * BATCH_KEYS) : null;
            value8 = records && approximate ? direct(8L * BATCH_KEYS) : null;
            vlen = records && approximate ? direct(BATCH_KEYS) : null;
            offs.putLong(0, 0L);
        }

        boolean fits(byte[] key, byte[] value) {
            return count < BATCH_KEYS && blob.position() + key.length <= blob.capacity();
        }

        void add(long a, byte[] key, byte[] value) {
            blob.put(key);
            offs.putLong(8 * (count + 1), blob.position());
            if (addr != null) addr.putLong(8 * count, a);
            if (value8 != null) {
                // index_a.db slot: the value's first min(len, 8) bytes (W:140-142); a
                // blocked writer's large record hands null (BlockedKVWriter.java:105-109)
                long v = 0;
                final int len = value == null ? 0 : Math.min(value.length, 8);
                for (int i = 0; i < len; i++) v |= (value[i] & 0xFFL) << (8 * i);
                value8.putLong(8 * count, v);
                vlen.put(count, (byte) len);
            }
            count++;
        }

        void flushKeys(long builder) {
            if (count > 0) GpuBuild.builderAddVar(builder, address(blob), address(offs), count, 0, 0, 0);
            reset();
        }

        void flushRecords(long ix, Object lock) {
            if (count > 0) {
                synchronized (lock) {  // one index writer: its puts in turn
                    GpuBuild.indexPutVar(ix, address(blob), address(offs), count, address(addr), address(value8),
                            address(vlen));
                }
            }
            reset();
        }

        private void reset() {
            count = 0;
            blob.clear();
        }

        private static ByteBuffer direct(long bytes) {
            return ByteBuffer.allocateDirect((int) bytes).order(ByteOrder.nativeOrder());
        }

        private static long address(ByteBuffer b) {  // null: no buffer (the C ABI takes NULL)
            return b == null ? 0L : ((DirectBuffer) b).address();
        }
    }
}

// jni/GpuBuild.java -- the Java side of the MI355X build path: one static
// native per C entry point of include/bsdb_mi355x.h that a JVM host needs
// (host-buffer forms; a JVM never holds device memory).  Conventions of the
// reference's own JNI class (src/main/java/tech/bsdb/io/Native.java:12-14,
// 147-156): the library is loaded from the jar, native objects cross as long,
// negative return codes become IOException (NativeFileIO.java:16-21).
// Not compiled here: this image and the GPU box have no JDK (INTEGRATION.md).
package tech.bsdb.gpu;

import tech.bsdb.io.NativeUtils;

public final class GpuBuild {
    static { NativeUtils.loadLibraryFromJar(System.mapLibraryName("bsdbgpujni")); }

    // context (bsdb_open/close) and knobs
    public static native long open(int device);
    public static native void close(long ctx);
    public static native long numBuckets(long n);                                   // GOV:281,350
    public static native long valuesWords(long n);                                  // GOV:357
    public static native void setVerify(long ctx, boolean on);
    public static native void releaseWorkspace(long ctx);                           // HBM back between builds
    // A3/A4/A6 from host memory (what put() batches feed)
    public static native void histogramFixed(long ctx, long keys, int keyLen, long n, long seed, long m, long counts);
    public static native void histogramVar(long ctx, long blob, long offs, long n, long seed, long m, long counts);
    public static native void hashFixed(long ctx, long keys, int keyLen, long n, long seed, long sig);
    public static native void hashVar(long ctx, long blob, long offs, long n, long seed, long sig);
    // B4: the histogram collective, one JVM per GPU (id shipped by the host's own channel)
    public static native byte[] commUniqueId();
    public static native void commInit(long ctx, int nranks, int rank, byte[] id);
    // B4: every GPU of this JVM (the reference's single-process build)
    public static native long multiOpen(int[] devices);
    public static native void multiClose(long mc);
    public static native void multiHistogramFixed(long mc, long keys, int keyLen, long n, long seed, long outE);
    public static native void multiHistogramVar(long mc, long blob, long offs, long n, long seed, long outE);
    // E4: the whole build (MPHF fields + index files) over every GPU of this JVM
    public static native void multiMphBuildIndexVar(long mc, long blob, long offs, long n, int checksumBits, long addr,
                                                    long value8, long vlen, boolean approximate, String indexPath,
                                                    String indexAPath, long outE, long outValues, long outSigBits);
    public static native void multiMphBuildIndexFixed(long mc, long keys, int keyLen, long n, int checksumBits,
                                                      long addr, long value8, long vlen, boolean approximate,
                                                      String indexPath, String indexAPath, long outE, long outValues,
                                                      long outSigBits);
    // A5-A11: the MPHF (F1) and its fields (A14), raw dump (A15), lookups (F4)
    public static native long mphBuildFixed(long ctx, long keys, int keyLen, long n, int checksumBits);
    public static native long mphBuildVar(long ctx, long blob, long offs, long n, int checksumBits);
    // F2: buildHash + buildIndex in one call (index from the solve's ranks, no kv.db rescan)
    public static native long mphBuildIndexVar(long ctx, long blob, long offs, long n, int checksumBits, long addr,
                                               long value8, long vlen, boolean approximate, String indexPath,
                                               String indexAPath);
    public static native long mphBuildIndexFixed(long ctx, long keys, int keyLen, long n, int checksumBits, long addr,
                                                 long value8, long vlen, boolean approximate, String indexPath,
                                                 String indexAPath);
    // F2 in bounded device memory: README-size sets on one GPU by bucket-range passes; addr 0 = the
    // records' addresses are addrBase + addrStride * i; passesOut[0] receives the passes used
    public static native long mphBuildIndexPassesFixed(long ctx, long keys, int keyLen, long n, int checksumBits,
                                                       long addr, long addrBase, long addrStride, long value8,
                                                       long vlen, boolean approximate, int passes, String indexPath,
                                                       String indexAPath, long[] passesOut);
    public static native long mphBuildIndexPassesVar(long ctx, long blob, long offs, long n, int checksumBits,
                                                     long addr, long addrBase, long addrStride, long value8,
                                                     long vlen, boolean approximate, int passes, String indexPath,
                                                     String indexAPath, long[] passesOut);
    // put() batches straight into HBM (CBHS.add, W:75-89), then buildHash + buildIndex in one finish
    public static native long builderOpen(long ctx, int keyLen, long keyCapacity, long blobCapacity,
                                          boolean approximate, long addrBase, long addrStride);
    public static native void builderAddFixed(long b, long keys, int keyLen, long count, long addr, long value8,
                                              long vlen);
    public static native void builderAddVar(long b, long blob, long offs, long count, long addr, long value8,
                                            long vlen);
    public static native long builderCount(long b);
    public static native long builderFinish(long b, int checksumBits, int passes, String indexPath, String indexAPath);
    public static native void builderFree(long b);
    public static native long[] mphInfo(long mph);        // {n, numBuckets, width, valuesWords, sigWords}
    public static native void mphExport(long mph, long outE, long outValues, long outSigBits);
    // {numBuckets, valuesWords, valueBits, sigWords} of an MPHF on n keys, no handle needed (GOV:350-357,494)
    public static native long[] mphSizes(long n, int checksumBits);
    // the export into Java arrays of the mphInfo sizes (sigBits null when checksumBits == 0): GovAssembler
    public static native void mphExportArrays(long mph, long[] outE, long[] outValues, long[] outSigBits);
    public static native long mphImport(long ctx, long n, int width, long E, long values, long sigBits);
    public static native void mphDump(long mph, String path);
    public static native long mphLoad(long ctx, String path);
    public static native void mphLookupFixed(long mph, long keys, int keyLen, long n, boolean check, long out);
    public static native void mphLookupVar(long mph, long blob, long offs, long n, boolean check, long out);
    public static native void mphFree(long mph);
    // A13: buildIndex (W:107-155)
    public static native long indexOpen(long mph, boolean approximate, long passCacheSize, String indexPath,
                                        String indexAPath, long[] passesOut);
    public static native void indexBeginPass(long ix, long pass);
    public static native void indexPutVar(long ix, long blob, long offs, long count, long addr, long value8, long vlen);
    public static native void indexPutFixed(long ix, long keys, int keyLen, long count, long addr, long value8, long vlen);
    public static native void indexEndPass(long ix);
    public static native void indexClose(long ix);
    // F3: build() straight from the data files: native kv.db scan (compact = 0 / blocked = 1 layouts)
    // + the one-call build; returns the MPHF handle (export it for hash.db as buildHash does)
    public static native long kvBuildIndex(long ctx, String kvBase, int partitions, int format, int blockSize,
                                           int threads, int checksumBits, boolean approximate, String indexPath,
                                           String indexAPath);
}

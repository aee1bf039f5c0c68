// jni/GovAssembler.java -- turns a device-built MPHF (bsdb_mph, exported
// through GpuBuild) into the reference's own hash-function object, so that
// BinIO.storeObject writes hash.db in the unchanged format Reader loads
// (src/main/java/tech/bsdb/read/Reader.java:30).
//
// The object is an instance of the reference's (modified, in-tree) class
// it.unimi.dsi.sux4j.mph.GOVMinimalPerfectHashFunctionModified, NOT a subclass:
// a subclass would put its own name into the serialized stream.  That class
// has one constructor, which builds the function itself from a bucketed hash
// store (GOV:329-516).  The fields it leaves behind are filled here instead,
// the way Java deserialization fills them: an instance from the constructor
// ReflectionFactory makes for serialization (no constructor of the class or
// its serializable superclasses runs), then every field of GOV:284-313 set
// from the exported arrays:
//   n                  the key count                        (GOV:345)
//   multiplier         2 * numBuckets                       (GOV:350-351)
//   globalSeed         0: BSDBWriter's store is never reseeded (CBHS:209, GOV:482)
//   edgeOffsetAndSeed  E, numBuckets + 1 longs: key offsets, local seed in the top byte (GOV:355,434-436)
//   bitVector          the 2-bit values, length 2 (V + 1) bits (GOV:357,483-485)
//   values             bitVector.asLongBigList(2)           (GOV:483)
//   array              bitVector.bits() (transient)         (GOV:485, readObject GOV:587-590)
//   transform          TransformationStrategies.byteArray() (W:43)
//   signatureMask      -1L >>> -w, or 0 with no signatures  (GOV:493,510)
//   signatures         n w-bit entries, or null             (GOV:494,511)
//   defRetValue        -1                                   (GOV:346)
// The sizes come from GpuBuild.mphSizes (bsdb_mph_sizes, the same arithmetic,
// tests/test_capi.py::test_mph_sizes_equal_gov_field_arithmetic).
//
// Not compiled here: this image and the GPU box have no JDK (INTEGRATION.md);
// tests/test_jni_shim.py checks that every simple name resolves.
package tech.bsdb.gpu;

import it.unimi.dsi.bits.LongArrayBitVector;
import it.unimi.dsi.bits.TransformationStrategies;
import it.unimi.dsi.sux4j.mph.GOVMinimalPerfectHashFunctionModified;
import sun.reflect.ReflectionFactory;

import java.io.IOException;
import java.lang.reflect.Constructor;
import java.lang.reflect.Field;

public final class GovAssembler {
    private GovAssembler() {
    }

    /** The hash function of a device MPHF handle (GpuBuild.mphBuild*, builderFinish, kvBuildIndex). */
    public static GOVMinimalPerfectHashFunctionModified<byte[]> fromMph(long mph) throws IOException {
        final long[] info = GpuBuild.mphInfo(mph);                 // {n, numBuckets, width, valuesWords, sigWords}
        final long n = info[0];
        final int width = (int) info[2];
        final long[] sizes = GpuBuild.mphSizes(n, width);         // {numBuckets, valuesWords, valueBits, sigWords}
        if (sizes[0] != info[1] || sizes[1] != info[3] || sizes[3] != info[4])
            throw new IOException("MPHF sizes disagree with GOV's arithmetic");
        final long[] E = new long[arrayLength(info[1] + 1)];
        final long[] values = new long[arrayLength(info[3])];
        final long[] sig = width == 0 ? null : new long[arrayLength(info[4])];
        GpuBuild.mphExportArrays(mph, E, values, sig);
        return assemble(n, E, values, sizes[2], width, sig);
    }

    /** The object from exported fields (E, the value words of valueBits bits, the checksum words). */
    public static GOVMinimalPerfectHashFunctionModified<byte[]> assemble(long n, long[] E, long[] valueWords,
                                                                        long valueBits, int width, long[] sigWords)
            throws IOException {
        if (E.length < 2 || (width != 0 && sigWords == null) || width < 0 || width > 64)
            throw new IllegalArgumentException("bad MPHF fields");
        final GOVMinimalPerfectHashFunctionModified<byte[]> f = blank();
        final LongArrayBitVector bitVector = LongArrayBitVector.wrap(valueWords, valueBits);
        set(f, "n", n);
        set(f, "multiplier", 2L * (E.length - 1));
        set(f, "globalSeed", 0L);
        set(f, "edgeOffsetAndSeed", E);
        set(f, "bitVector", bitVector);
        set(f, "values", bitVector.asLongBigList(2));
        set(f, "array", bitVector.bits());
        set(f, "transform", TransformationStrategies.byteArray());
        if (width == 0) {
            set(f, "signatureMask", 0L);
            set(f, "signatures", null);
        } else {
            set(f, "signatureMask", -1L >>> -width);
            set(f, "signatures", LongArrayBitVector.wrap(sigWords, n * width).asLongBigList(width));
        }
        f.defaultReturnValue(-1);
        return f;
    }

    @SuppressWarnings("unchecked")
    private static GOVMinimalPerfectHashFunctionModified<byte[]> blank() throws IOException {
        try {
            final Constructor<?> c = ReflectionFactory.getReflectionFactory().newConstructorForSerialization(
                    GOVMinimalPerfectHashFunctionModified.class, Object.class.getDeclaredConstructor());
            return (GOVMinimalPerfectHashFunctionModified<byte[]>) c.newInstance();
        } catch (ReflectiveOperationException e) {
            throw new IOException("cannot instantiate the hash function class", e);
        }
    }

    private static void set(Object f, String name, Object value) throws IOException {
        try {
            final Field field = GOVMinimalPerfectHashFunctionModified.class.getDeclaredField(name);
            field.setAccessible(true);
            field.set(f, value);
        } catch (ReflectiveOperationException e) {
            throw new IOException("cannot set field " + name, e);
        }
    }

    private static int arrayLength(long words) throws IOException {
        if (words > Integer.MAX_VALUE - 8) throw new IOException(words + " words do not fit one Java array");
        return (int) words;
    }
}

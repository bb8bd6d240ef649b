package com.covt.decoder.gpu;

import com.covt.decoder.DecodingUtils;
import me.lemire.integercompression.IntWrapper;

/**
 * Drop-in replacement for com.covt.decoder.DecodingUtils whose methods decode on an AMD MI355X
 * through libcovt (include/covt.h) and the JNI shim cov-tiles_amd/jni/covt_jni.cc.  Signatures and
 * cursor semantics are those of DecodingUtils.java:35-444; errors surface as the same exception
 * types (IllegalArgumentException, ArrayIndexOutOfBoundsException).  Every DecodingUtils method that
 * CovtParser.decodeCovt reaches is here: the integer decoders run on the GPU; decodeFloatsLE and
 * decodeString (byte views with no decode arithmetic) pass through to DecodingUtils.
 */
public final class GpuDecodingUtils {
    static { System.loadLibrary("covt_jni"); }

    private GpuDecodingUtils() {}

    public static native int[] decodeVarint(byte[] src, IntWrapper pos, int numValues);

    public static native int[] decodeZigZagVarint(byte[] src, IntWrapper pos, int numValues);

    public static native int[] decodeZigZagDeltaVarint(byte[] src, IntWrapper pos, int numValues);

    public static native int[] decodeZigZagDeltaVarintCoordinates(byte[] src, IntWrapper pos, int numValues);

    public static native long[] decodeRle(byte[] buffer, int numValues, IntWrapper pos, boolean signed);

    public static native byte[] decodeByteRle(byte[] buffer, int numValues, IntWrapper pos, int byteLength);

    /** DecodingUtils.java:290 -- advances by the ORC re-encoded length (CovtParser.java:295, Gen D present). */
    public static byte[] decodeByteRle(byte[] buffer, int numValues, IntWrapper pos) {
        return decodeByteRleReencode(buffer, numValues, pos);
    }

    private static native byte[] decodeByteRleReencode(byte[] buffer, int numValues, IntWrapper pos);

    /** DecodingUtils.java:446 (CovtParser.java:328): a little-endian view of the bytes, no decode arithmetic. */
    public static float[] decodeFloatsLE(byte[] encodedValues, IntWrapper pos, int numValues) {
        return DecodingUtils.decodeFloatsLE(encodedValues, pos, numValues);
    }

    /** DecodingUtils.java:21 (CovtParser.java:386): varint length + UTF-8 bytes, host work. */
    public static String decodeString(byte[] content, IntWrapper pos) {
        return DecodingUtils.decodeString(content, pos);
    }

    /** DecodingUtils.java:28. */
    public static String decodeString(byte[] content, IntWrapper pos, int numChars) {
        return DecodingUtils.decodeString(content, pos, numChars);
    }

    public static native int[] decodeFastPfor128ZigZagDelta(byte[] encodedValues, int numValues, int byteLength,
                                                            IntWrapper pos);

    public static native int[] decodeFastPfor128DeltaCoordinates(byte[] encodedValues, int numValues,
                                                                 int byteLength, IntWrapper pos);

    public static native int[] decodeDeltaVarintMortonCodes(byte[] src, IntWrapper pos, int numVertices,
                                                            int numBits);

    public static native int[] decodeFastPfor128DeltaMortonCodes(byte[] encodedValues, int numVertices,
                                                                 int byteLength, IntWrapper pos, int numBits);
}

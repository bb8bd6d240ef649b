package com.covt.decoder.gpu;

import me.lemire.integercompression.IntWrapper;

/**
 * Drop-in replacement for com.covt.decoder.DecodingUtils whose methods decode on an AMD MI355X
 * through libcovt (include/covt.h) and the JNI shim cov-tiles_amd/jni/covt_jni.cc.  Signatures and
 * cursor semantics are those of DecodingUtils.java:35-444; errors surface as the same exception
 * types (IllegalArgumentException, ArrayIndexOutOfBoundsException).
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

    public static native int[] decodeFastPfor128ZigZagDelta(byte[] encodedValues, int numValues, int byteLength,
                                                            IntWrapper pos);

    public static native int[] decodeFastPfor128DeltaCoordinates(byte[] encodedValues, int numValues,
                                                                 int byteLength, IntWrapper pos);

    public static native int[] decodeDeltaVarintMortonCodes(byte[] src, IntWrapper pos, int numVertices,
                                                            int numBits);

    public static native int[] decodeFastPfor128DeltaMortonCodes(byte[] encodedValues, int numVertices,
                                                                 int byteLength, IntWrapper pos, int numBits);
}

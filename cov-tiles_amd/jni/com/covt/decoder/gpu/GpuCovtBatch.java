package com.covt.decoder.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;

/**
 * Whole-tile batch decode on an AMD MI355X through libcovt's plan API (include/covt.h, "plan"):
 * the metadata of every tile is walked on the host (what CovtParser.decodeCovt does per layer,
 * CovtParser.java:53-133), then every Id and Geometry stream -- and with PLAN_PROPERTIES every
 * property column -- of the whole batch is decoded in one GPU launch.  Outputs land in direct
 * ByteBuffers (little-endian) at the offsets of {@link #streams()} / {@link #propertyColumns()},
 * so a Java caller reads them without copies; per-stream statuses are the include/covt.h codes.
 *
 * <p>Built with the JNI shim cov-tiles_amd/jni/covt_jni.cc (make -C cov-tiles_amd jni JAVA_HOME=...).
 */
public final class GpuCovtBatch implements AutoCloseable {
    static { System.loadLibrary("covt_jni"); }

    public static final int FORMAT_GENC = 0;     // COVT_FORMAT_GENC: the committed fixtures
    public static final int FORMAT_GEND = 1;     // COVT_FORMAT_GEND: what CovtParser.decodeCovt reads
    public static final int ID_FORMAT = 0;       // COVT_ID_FORMAT: 64-bit ids
    public static final int ID_JAVA = 1;         // COVT_ID_JAVA: CovtParser's 4-byte varint cap
    public static final int PLAN_PROPERTIES = 1; // COVT_PLAN_PROPERTIES
    /** Fields per row of {@link #streams()}: covt_stream_info in order (tile, layer, column_kind,
     * stream_type, encoding, column_type, num_values, byte_length, num_bits, op, elem_bytes,
     * desc_index, in_off, out_off, out_elems). */
    public static final int STREAM_FIELDS = 15;
    /** Fields per row of {@link #propertyColumns()}: covt_prop_info in order (tile, layer, column, type,
     * column_type, n_features, n_data, n_dict, lang, name_len, lang_len, dict_bytes, stream[3],
     * desc_index, name_off, lang_off, out_off[4]); name_off / lang_off index the batch input. */
    public static final int PROPERTY_FIELDS = 22;

    private final ByteBuffer tiles;
    private final int numTiles;
    private long handle;

    public GpuCovtBatch(byte[][] tileBytes, int format, int idMode, int flags) {
        long total = 0;
        for (byte[] t : tileBytes) total += t.length;
        if (total > Integer.MAX_VALUE) throw new IllegalArgumentException("batch larger than 2 GiB");
        tiles = ByteBuffer.allocateDirect((int) total).order(ByteOrder.LITTLE_ENDIAN);
        long[] offsets = new long[tileBytes.length];
        long[] sizes = new long[tileBytes.length];
        for (int i = 0; i < tileBytes.length; i++) {
            offsets[i] = tiles.position();
            sizes[i] = tileBytes[i].length;
            tiles.put(tileBytes[i]);
        }
        tiles.clear();
        numTiles = tileBytes.length;
        handle = create(tiles, offsets, sizes, format, idMode, flags);
    }

    /** Per-tile walk status (0, or a negative COVT_ERR_*: that tile has no streams). */
    public int[] tileStatus() { return tileStatus(live(), numTiles); }

    public long numStreams() { return numStreams(live()); }

    /** Bytes {@link #decode} writes. */
    public long outputBytes() { return outputBytes(live()); }

    /** numStreams() rows of STREAM_FIELDS values, plan stream (tile) order. */
    public long[] streams() { return streams(live()); }

    /** Decodes every planned stream into {@code out} (direct, outputBytes() long); returns one
     * status per stream, plan order (COVT_OK = 0). */
    public int[] decode(ByteBuffer out) {
        if (!out.isDirect() || out.capacity() < outputBytes()) throw new IllegalArgumentException("output buffer");
        return decode(live(), tiles, out);
    }

    public long numPropertyColumns() { return numPropertyColumns(live()); }

    /** Bytes {@link #properties} writes. */
    public long propertyBytes() { return propertyBytes(live()); }

    /** numPropertyColumns() rows of PROPERTY_FIELDS values, tile order. */
    public long[] propertyColumns() { return propertyColumns(live()); }

    /** Decode + property materialization into {@code out} (direct, propertyBytes() long); returns
     * (status, n_valid) per property column, tile order. */
    public int[] properties(ByteBuffer out) {
        if (!out.isDirect() || out.capacity() < propertyBytes()) throw new IllegalArgumentException("output buffer");
        return properties(live(), tiles, out);
    }

    @Override
    public void close() {
        if (handle != 0) destroy(handle);
        handle = 0;
    }

    private long live() {
        if (handle == 0) throw new IllegalStateException("closed");
        return handle;
    }

    private static native long create(ByteBuffer tiles, long[] offsets, long[] sizes, int format, int idMode, int flags);
    private static native void destroy(long plan);
    private static native int[] tileStatus(long plan, int numTiles);
    private static native long numStreams(long plan);
    private static native long outputBytes(long plan);
    private static native long[] streams(long plan);
    private static native int[] decode(long plan, ByteBuffer tiles, ByteBuffer out);
    private static native long numPropertyColumns(long plan);
    private static native long propertyBytes(long plan);
    private static native long[] propertyColumns(long plan);
    private static native int[] properties(long plan, ByteBuffer tiles, ByteBuffer out);
}

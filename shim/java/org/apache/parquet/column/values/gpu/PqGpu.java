/*
 * Entry points of the MI355X page decoder (libpqgpu.so via libpqgpu_jni.so) for parquet-mr code in
 * other packages (ParquetReadRouter lives in org.apache.parquet.column.values.bitpacking,
 * ColumnReaderBase in org.apache.parquet.column.impl): every method a caller needs is public.
 *
 * ByteBuffers may be direct or heap (parquet-mr's default allocator is HeapByteBufferAllocator,
 * ParquetReadOptions.java:265): the bytes from position() to limit() are used in both cases. A heap
 * buffer is passed as its backing array (array() + arrayOffset() + position()); a read-only heap
 * buffer is copied once. The natives below take (buffer or array, offset, length) and never look at
 * the buffer's position themselves.
 *
 * JNI glue: shim/jni/pqgpu_jni.c; C ABI: include/pqgpu.h, include/pqgpu_reader.h.
 */
package org.apache.parquet.column.values.gpu;

import java.nio.ByteBuffer;

public final class PqGpu {
  static {
    System.loadLibrary("pqgpu_jni");
  }

  private PqGpu() {}

  /** Size of one packed pqg_page_desc / pqg_column_desc (little endian, C layout). */
  public static final int PAGE_DESC_BYTES = 56;
  public static final int COLUMN_DESC_BYTES = 104;
  /** pqg_column_desc.flags: decode dictionary ids (readValueDictionaryId) instead of values. */
  public static final int COLUMN_DICTIONARY_IDS = 1;
  /** ColumnMetaData.codec values (parquet.thrift CompressionCodec; pqg_codec). */
  public static final int CODEC_UNCOMPRESSED = 0, CODEC_SNAPPY = 1, CODEC_GZIP = 2, CODEC_LZO = 3,
      CODEC_BROTLI = 4, CODEC_LZ4 = 5, CODEC_ZSTD = 6, CODEC_LZ4_RAW = 7;

  /** Number of visible MI355X devices (0: no GPU path; the caller keeps the CPU readers). */
  public static native int deviceCount();

  /** One decode context (HIP stream + device scratch); not thread-safe: one per reader thread. */
  public static native long ctxCreate(int device);

  public static native void ctxDestroy(long ctx);

  /** JNI class name of the exception for a pqg_error code (pqg_java_exception). */
  public static native String exceptionClass(int code);

  private static final ThreadLocal<long[]> THREAD_CTX = new ThreadLocal<long[]>();

  /**
   * The calling thread's context on device 0, created on first use (what a ParquetReadRouter branch
   * or a column reader uses; parquet-mr reads a row group's columns on one thread). Released by
   * {@link #releaseThreadContext()}.
   */
  public static long threadContext() {
    long[] c = THREAD_CTX.get();
    if (c == null) {
      c = new long[] {ctxCreate(0)};
      THREAD_CTX.set(c);
    }
    return c[0];
  }

  public static void releaseThreadContext() {
    long[] c = THREAD_CTX.get();
    if (c != null) {
      ctxDestroy(c[0]);
      THREAD_CTX.remove();
    }
  }

  /**
   * Page headers of one raw column chunk (ParquetFileReader.Chunk.readAllPages) in
   * chunk[position, limit): returns packed pqg_page_desc[] of its data pages, fills dictInfo = {dict
   * offset, size, num_values, encoding} (offset -1: none). codec = ColumnMetaData.codec: with a codec
   * other than CODEC_UNCOMPRESSED a V1 / dictionary page, or a V2 page with is_compressed set, throws
   * UnsupportedOperationException (decompress first). Throws ParquetDecodingException on a CRC
   * mismatch / corrupt header. Descriptor offsets are chunkOffset + offset inside the chunk.
   */
  public static byte[] frameChunk(ByteBuffer chunk, long valueCount, boolean verifyCrc, int codec, long chunkOffset,
      int column, long[] dictInfo) {
    if (chunk.isDirect()) {
      return frameChunkDirect(chunk, chunk.position(), chunk.remaining(), valueCount, verifyCrc, codec, chunkOffset,
          column, dictInfo);
    }
    byte[] a = heapBytes(chunk);
    int off = chunk.hasArray() && !chunk.isReadOnly() ? chunk.arrayOffset() + chunk.position() : 0;
    return frameChunkArray(a, off, chunk.remaining(), valueCount, verifyCrc, codec, chunkOffset, column, dictInfo);
  }

  /**
   * Decode every page of a batch in one call (the staged host path: pqg_host_input,
   * pqg_decode_staged, pqg_staged_column; no Java array is held while the device works);
   * pageBytes[position, limit) holds the bytes the descriptors' offsets refer to. values[i]: long[] /
   * int[] / float[] / double[] / byte[] (BOOLEAN, FIXED_LEN_BYTE_ARRAY, INT96 row-major) or long[]
   * offsets (n + 1) for BYTE_ARRAY (binary[i] receives the bytes), int[] for COLUMN_DICTIONARY_IDS
   * columns of any type; defLevels[i] / repLevels[i] receive the levels of columns with max level > 0.
   * An element that is null or too short is replaced by a new array of the exact decoded size (a
   * wrong element type throws IllegalArgumentException). pageCounts receives each page's value count.
   * Returns {code, page, value_index, 0, values_written[0..nCols), then per page (code, phase, index)
   * (pqg_page_errors)}. Decode errors are returned, not thrown: the readers throw them where the
   * reference readers would (GpuPageBatch).
   */
  public static long[] decodeHost(long ctx, ByteBuffer pageBytes, byte[] pageDescs, byte[] columnDescs, Object[] values,
      byte[][] defLevels, byte[][] repLevels, byte[][] binary, int[] pageCounts) {
    if (pageBytes.isDirect()) {
      return decodeHostDirect(ctx, pageBytes, pageBytes.position(), pageBytes.remaining(), pageDescs, columnDescs,
          values, defLevels, repLevels, binary, pageCounts);
    }
    byte[] a = heapBytes(pageBytes);
    int off = pageBytes.hasArray() && !pageBytes.isReadOnly() ? pageBytes.arrayOffset() + pageBytes.position() : 0;
    return decodeHostArray(ctx, a, off, pageBytes.remaining(), pageDescs, columnDescs, values, defLevels, repLevels,
        binary, pageCounts);
  }

  /**
   * ParquetReadRouter.read on the GPU (pqg_router_read): unpack `count` LSB-first values of
   * `bitWidth` bits from in[position, limit) (count * bitWidth / 8 bytes; fewer -> EOFException)
   * into out[0..count).
   */
  public static void routerRead(long ctx, int bitWidth, ByteBuffer in, int count, int[] out)
      throws java.io.EOFException {
    if (in.isDirect()) {
      routerReadDirect(ctx, bitWidth, in, in.position(), in.remaining(), count, out);
      return;
    }
    byte[] a = heapBytes(in);
    int off = in.hasArray() && !in.isReadOnly() ? in.arrayOffset() + in.position() : 0;
    routerReadArray(ctx, bitWidth, a, off, in.remaining(), count, out);
  }

  /**
   * A page's bit-packed runs in one call (pqg_router_read_runs): run r is ParquetReadRouter.read(bitWidth,
   * in positioned at position() + runOffsets[r], runCounts[r], ...), its values go to out after the
   * earlier runs' values. One PCIe round trip for the whole batch instead of one per run; a run whose
   * runCounts[r] * bitWidth / 8 bytes pass the buffer's limit -> EOFException before anything is written.
   */
  public static void routerReadBatch(long ctx, int bitWidth, ByteBuffer in, long[] runOffsets, int[] runCounts,
      int nRuns, int[] out) throws java.io.EOFException {
    if (in.isDirect()) {
      routerReadBatchDirect(ctx, bitWidth, in, in.position(), in.remaining(), runOffsets, runCounts, nRuns, out);
      return;
    }
    byte[] a = heapBytes(in);
    int off = in.hasArray() && !in.isReadOnly() ? in.arrayOffset() + in.position() : 0;
    routerReadBatchArray(ctx, bitWidth, a, off, in.remaining(), runOffsets, runCounts, nRuns, out);
  }

  /**
   * ParquetReadRouter.read with its contract kept (the run's values are in out[0..count) when the call
   * returns) at one device round trip per page (pqg_router_read_page). `tail` holds the caller's stream
   * from the run's data start to the stream's end in [position, limit): the first read of a page also
   * unpacks every later bit-packed run of the stream, and the reads of those runs are served from the
   * library's cache with no device work. The caller advances its own stream by count * bitWidth / 8
   * bytes; fewer bytes than that in `tail` -> EOFException with nothing written.
   */
  public static void routerReadPage(long ctx, int bitWidth, ByteBuffer tail, int count, int[] out)
      throws java.io.EOFException {
    if (tail.isDirect()) {
      routerReadPageDirect(ctx, bitWidth, tail, tail.position(), tail.remaining(), count, out);
      return;
    }
    byte[] a = heapBytes(tail);
    int off = tail.hasArray() && !tail.isReadOnly() ? tail.arrayOffset() + tail.position() : 0;
    routerReadPageArray(ctx, bitWidth, a, off, tail.remaining(), count, out);
  }

  /** The backing array of a heap buffer, or a copy of [position, limit) of a read-only one. */
  private static byte[] heapBytes(ByteBuffer b) {
    if (b.hasArray() && !b.isReadOnly()) return b.array();
    byte[] copy = new byte[b.remaining()];
    b.duplicate().get(copy);
    return copy;
  }

  private static native byte[] frameChunkDirect(ByteBuffer chunk, int offset, int length, long valueCount,
      boolean verifyCrc, int codec, long chunkOffset, int column, long[] dictInfo);

  private static native byte[] frameChunkArray(byte[] chunk, int offset, int length, long valueCount,
      boolean verifyCrc, int codec, long chunkOffset, int column, long[] dictInfo);

  private static native long[] decodeHostDirect(long ctx, ByteBuffer pageBytes, int offset, int length,
      byte[] pageDescs, byte[] columnDescs, Object[] values, byte[][] defLevels, byte[][] repLevels, byte[][] binary,
      int[] pageCounts);

  private static native long[] decodeHostArray(long ctx, byte[] pageBytes, int offset, int length, byte[] pageDescs,
      byte[] columnDescs, Object[] values, byte[][] defLevels, byte[][] repLevels, byte[][] binary, int[] pageCounts);

  private static native void routerReadDirect(long ctx, int bitWidth, ByteBuffer in, int offset, int length, int count,
      int[] out);

  private static native void routerReadArray(long ctx, int bitWidth, byte[] in, int offset, int length, int count,
      int[] out);

  private static native void routerReadPageDirect(long ctx, int bitWidth, ByteBuffer tail, int offset, int length,
      int count, int[] out);

  private static native void routerReadPageArray(long ctx, int bitWidth, byte[] tail, int offset, int length,
      int count, int[] out);

  private static native void routerReadBatchDirect(long ctx, int bitWidth, ByteBuffer in, int offset, int length,
      long[] runOffsets, int[] runCounts, int nRuns, int[] out);

  private static native void routerReadBatchArray(long ctx, int bitWidth, byte[] in, int offset, int length,
      long[] runOffsets, int[] runCounts, int nRuns, int[] out);
}

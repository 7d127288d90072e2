/*
 * Native entry points of the MI355X page decoder (libpqgpu.so via libpqgpu_jni.so).
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
  public static final int PAGE_DESC_BYTES = 48;
  public static final int COLUMN_DESC_BYTES = 104;
  /** pqg_column_desc.flags: decode dictionary ids (readValueDictionaryId) instead of values. */
  public static final int COLUMN_DICTIONARY_IDS = 1;

  /** Number of visible MI355X devices (0: no GPU path; the caller keeps the CPU readers). */
  static native int deviceCount();

  /** One decode context (HIP stream + device scratch) per reader thread, like ColumnReaderBase. */
  static native long ctxCreate(int device);

  static native void ctxDestroy(long ctx);

  /**
   * Page headers of one raw column chunk (ParquetFileReader.Chunk.readAllPages): returns packed
   * pqg_page_desc[] of its data pages, fills dictInfo = {dict offset, size, num_values, encoding}
   * (offset -1: none). Throws ParquetDecodingException on a CRC mismatch / corrupt header.
   */
  static native byte[] frameChunk(ByteBuffer chunk, long valueCount, boolean verifyCrc, long chunkOffset, int column,
      long[] dictInfo);

  /**
   * Decode every page of a batch in one call (pqg_decode_host). values[i]: long[] / int[] / float[] /
   * double[] / byte[] (BOOLEAN, FIXED_LEN_BYTE_ARRAY, INT96 row-major) or long[] offsets for
   * BYTE_ARRAY (binary[i] receives the bytes), int[] for COLUMN_DICTIONARY_IDS columns; defLevels /
   * repLevels may hold null. pageCounts receives each page's value count. Returns {code, page,
   * value_index, kind (0 none, 1 value error: lazily at that read, 2 page error: at initFromPage),
   * values_written[0..nCols)}. Decode errors are returned, not thrown: the readers throw them where
   * the reference readers would.
   */
  static native long[] decodeHost(long ctx, ByteBuffer pageBytes, byte[] pageDescs, byte[] columnDescs,
      Object[] values, byte[][] defLevels, byte[][] repLevels, byte[][] binary, int[] pageCounts);

  /**
   * ParquetReadRouter.read on the GPU (pqg_router_read): unpack `count` LSB-first values of `bitWidth`
   * bits from the direct buffer `in` (count * bitWidth / 8 bytes) into out[0..count).
   */
  static native void routerRead(long ctx, int bitWidth, ByteBuffer in, int count, int[] out);

  /** JNI class name of the exception for a pqg_error code (pqg_java_exception). */
  static native String exceptionClass(int code);
}

/*
 * Repetition or definition levels of one page, decoded on the GPU: the level reader
 * ColumnReaderBase.readPageV1 builds (RunLengthBitPackingHybridValuesReader,
 * parquet-column/src/main/java/org/apache/parquet/column/values/rle/RunLengthBitPackingHybridValuesReader.java:40-65;
 * ByteBitPackingValuesReader for BIT_PACKED; ZeroIntegerValuesReader when the max level is 0) and the
 * RLEIntIterator / NullIntIterator of readPageV2 (ColumnReaderBase.java:760-789), served from the
 * batch's u8 level array. Same state machine as pqg_levels_reader (include/pqgpu_reader.h,
 * parquet-mr_amd/csrc/pqgpu_reader.cpp), which tests/c/harness.c pins.
 *
 * ColumnReaderBase wraps it as it wraps the CPU readers: new ValuesReaderIntIterator(reader), whose
 * nextInt() calls readInteger() (INTEGRATION.md §1).
 */
package org.apache.parquet.column.values.gpu;

import java.io.IOException;
import org.apache.parquet.bytes.ByteBufferInputStream;
import org.apache.parquet.column.values.ValuesReader;
import org.apache.parquet.io.ParquetDecodingException;

public final class GpuLevelsReader extends ValuesReader {
  private final GpuPageBatch batch;
  private final byte[] levels; // null: max level 0 (every read is 0)
  private final long end;
  private final long errorAt;
  private final int errorCode;
  private long pos;

  GpuLevelsReader(GpuPageBatch batch, byte[] levels, long first, long end, int errorCode, long errorAt) {
    this.batch = batch;
    this.levels = levels;
    this.pos = first;
    this.end = end;
    this.errorCode = errorCode;
    this.errorAt = errorAt;
  }

  /**
   * The levels were decoded on the device: nothing of the page's stream is consumed here (the
   * GpuValuesReader of the same page consumes the whole remaining section), so readPageV1's
   * rlReader / dlReader / data reader sequence over one stream stays valid.
   */
  @Override
  public void initFromPage(int valueCount, ByteBufferInputStream in) throws IOException {}

  /** Slots left in the page. */
  public long remaining() {
    return Math.max(0, end - pos);
  }

  @Override
  public int readInteger() {
    if (errorCode != 0 && pos >= errorAt) throw batch.exception(errorCode, "level of slot " + pos);
    if (levels == null) { // ZeroIntegerValuesReader / NullIntIterator
      pos++;
      return 0;
    }
    if (pos >= end) throw new ParquetDecodingException("no more levels in the page");
    return levels[(int) pos++] & 0xFF;
  }

  @Override
  public void skip() {
    readInteger();
  }
}

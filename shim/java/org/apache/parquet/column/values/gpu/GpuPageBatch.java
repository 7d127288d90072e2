/*
 * The pages of one or more column chunks decoded in one native call: what ColumnReaderBase reads
 * page by page (ColumnReaderBase.readPageV1/V2, ColumnReaderBase.java:738-789) is decoded up front
 * on the GPU; each page then gets a GpuValuesReader over its slice of the dense column and two
 * GpuLevelsReaders over its slots' repetition / definition levels.
 *
 * Errors are scoped the way the reference scopes them: a ColumnReader fails on its own
 * (ColumnReaderBase.java:590-623, 650-676) and the other columns of the batch stay readable. Each
 * page carries its own first error (pqg_page_errors); a reader of page p throws where the reference's
 * reader of p throws, and every reader of a later page of the same column throws at init (that
 * column's reader never got past p). Same rules as include/pqgpu_reader.h, pinned by
 * tests/c/harness.c.
 */
package org.apache.parquet.column.values.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import org.apache.parquet.io.ParquetDecodingException;

public final class GpuPageBatch {
  /** pqg_phase (include/pqgpu.h). */
  static final int PHASE_DICTIONARY = 1, PHASE_RL_INIT = 2, PHASE_DL_INIT = 3, PHASE_DATA_INIT = 4,
      PHASE_RL_READ = 5, PHASE_DL_READ = 6, PHASE_VALUE = 7;

  final Object[] values;
  final byte[][] defLevels;
  final byte[][] repLevels;
  final byte[][] binary;
  final int[] physicalType;
  final int[] typeLength;
  final int[] flags;
  final int[] maxRep;
  final int[] maxDef;
  final long[] valuesWritten;
  private final int[] pageCounts;
  private final int[] pageColumn;
  private final long[] pageFirstValue;
  private final long[] pageFirstSlot;
  private final int[] pageSlots;
  private final int[] errCode;
  private final int[] errPhase;
  private final long[] errIndex;
  /** Per page: the code of an earlier failing page of its column (0: none). */
  private final int[] failedBefore;

  /**
   * @param pageBytes direct or heap buffer; [position, limit) holds every page body (and dictionary
   *     page) the descriptors refer to (descriptor offsets are relative to position)
   * @param pageDescs packed pqg_page_desc[] (PqGpu.frameChunk output, concatenated per chunk)
   * @param columnDescs packed pqg_column_desc[] (output fields unused)
   * @param values / defLevels / repLevels / binary per column: arrays to fill, or null elements for the
   *     native side to allocate at the exact decoded size (it stores them back into these arrays)
   */
  public GpuPageBatch(long ctx, ByteBuffer pageBytes, byte[] pageDescs, byte[] columnDescs, Object[] values,
      byte[][] defLevels, byte[][] repLevels, byte[][] binary) {
    int nPages = pageDescs.length / PqGpu.PAGE_DESC_BYTES;
    int nCols = columnDescs.length / PqGpu.COLUMN_DESC_BYTES;
    this.values = values;
    this.defLevels = defLevels;
    this.repLevels = repLevels;
    this.binary = binary;
    this.pageCounts = new int[nPages];
    ByteBuffer cd = ByteBuffer.wrap(columnDescs).order(ByteOrder.LITTLE_ENDIAN);
    physicalType = new int[nCols];
    typeLength = new int[nCols];
    flags = new int[nCols];
    maxRep = new int[nCols];
    maxDef = new int[nCols];
    for (int i = 0; i < nCols; i++) {
      int b = i * PqGpu.COLUMN_DESC_BYTES;
      physicalType[i] = cd.getInt(b);
      typeLength[i] = cd.getInt(b + 4);
      maxRep[i] = cd.getInt(b + 8);
      maxDef[i] = cd.getInt(b + 12);
      flags[i] = cd.getInt(b + 36);
    }
    long[] r = PqGpu.decodeHost(ctx, pageBytes, pageDescs, columnDescs, values, defLevels, repLevels, binary,
        pageCounts);
    valuesWritten = new long[nCols];
    System.arraycopy(r, 4, valuesWritten, 0, nCols);
    errCode = new int[nPages];
    errPhase = new int[nPages];
    errIndex = new long[nPages];
    for (int p = 0; p < nPages; p++) {
      int b = 4 + nCols + 3 * p;
      errCode[p] = (int) r[b];
      errPhase[p] = (int) r[b + 1];
      errIndex[p] = r[b + 2];
    }
    // one pass: each page's column, first value, first slot, and its column's earlier failure
    ByteBuffer pd = ByteBuffer.wrap(pageDescs).order(ByteOrder.LITTLE_ENDIAN);
    pageColumn = new int[nPages];
    pageFirstValue = new long[nPages];
    pageFirstSlot = new long[nPages];
    pageSlots = new int[nPages];
    failedBefore = new int[nPages];
    long[] accV = new long[Math.max(nCols, 1)];
    long[] accS = new long[Math.max(nCols, 1)];
    int[] colFail = new int[Math.max(nCols, 1)];
    for (int p = 0; p < nPages; p++) {
      int base = p * PqGpu.PAGE_DESC_BYTES;
      int c = pd.getInt(base + 16);
      pageColumn[p] = c;
      pageSlots[p] = pd.getInt(base + 12);
      if (c >= 0 && c < nCols) {
        pageFirstValue[p] = accV[c];
        pageFirstSlot[p] = accS[c];
        failedBefore[p] = colFail[c];
        accV[c] += pageCounts[p];
        accS[c] += pageSlots[p] & 0xFFFFFFFFL;
        if (colFail[c] == 0) colFail[c] = errCode[p];
      }
    }
  }

  public int pageCount() {
    return pageColumn.length;
  }

  /** The data reader of one page (the ValuesReader ColumnReaderBase.initDataReader would create). O(1). */
  public GpuValuesReader reader(int page) {
    int column = pageColumn[page];
    long first = pageFirstValue[page];
    if (failedBefore[page] != 0) throw exception(failedBefore[page], "column " + column + " failed on an earlier page");
    long errorAt = -1;
    if (errCode[page] != 0) {
      switch (errPhase[page]) {
        case PHASE_VALUE:
          errorAt = first + errIndex[page];
          break;
        case PHASE_RL_READ:
        case PHASE_DL_READ:
          break; // the page's values stop at the slots before the level error
        default:
          throw exception(errCode[page], "page " + page + " of the batch cannot be read");
      }
    }
    return new GpuValuesReader(this, column, first, first + pageCounts[page], errCode[page], errorAt);
  }

  /** The repetition-level reader of one page (readPageV1's rlReader / readPageV2's repetitionLevelColumn). */
  public GpuLevelsReader repLevels(int page) {
    return levels(page, true);
  }

  /** The definition-level reader of one page (readPageV1's dlReader / readPageV2's definitionLevelColumn). */
  public GpuLevelsReader defLevels(int page) {
    return levels(page, false);
  }

  private GpuLevelsReader levels(int page, boolean rep) {
    int column = pageColumn[page];
    if (failedBefore[page] != 0) throw exception(failedBefore[page], "column " + column + " failed on an earlier page");
    long first = pageFirstSlot[page];
    long end = first + (pageSlots[page] & 0xFFFFFFFFL);
    int code = 0;
    long errorAt = -1;
    if (errCode[page] != 0) {
      switch (errPhase[page]) {
        case PHASE_DICTIONARY:
        case PHASE_RL_INIT: // readPageV1: the rl reader's init throws, no dl reader is created
          throw exception(errCode[page], "page " + page + " levels cannot be read");
        case PHASE_DL_INIT:
          if (!rep) throw exception(errCode[page], "page " + page + " definition levels cannot be read");
          break;
        case PHASE_RL_READ: // rl(s) throws; dl(s) is never read
          code = errCode[page];
          errorAt = first + errIndex[page];
          break;
        case PHASE_DL_READ: // rl(s) was read, dl(s) throws
          code = errCode[page];
          errorAt = first + errIndex[page] + (rep ? 1 : 0);
          break;
        default:
          break;
      }
    }
    byte[][] arrays = rep ? repLevels : defLevels;
    int maxLevel = rep ? maxRep[column] : maxDef[column];
    byte[] lv = maxLevel > 0 && arrays != null ? arrays[column] : null;
    if (maxLevel > 0 && lv == null) throw new IllegalStateException("levels of column " + column + " were not decoded");
    return new GpuLevelsReader(this, lv, first, end, code, errorAt);
  }

  RuntimeException exception(int c, String what) {
    String cls = PqGpu.exceptionClass(c);
    String msg = what + " (pqg error " + c + ")";
    if (cls == null) return new ParquetDecodingException(msg);
    switch (cls) {
      case "java/lang/UnsupportedOperationException":
        return new UnsupportedOperationException(msg);
      case "java/lang/ArrayIndexOutOfBoundsException":
        return new ArrayIndexOutOfBoundsException(msg);
      case "java/lang/IllegalArgumentException":
        return new IllegalArgumentException(msg);
      case "java/lang/IllegalStateException":
        return new IllegalStateException(msg);
      default:
        return new ParquetDecodingException(msg);
    }
  }
}

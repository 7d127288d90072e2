/*
 * The pages of one or more column chunks decoded in one native call: what ColumnReaderBase reads
 * page by page (ColumnReaderBase.readPageV1/V2, ColumnReaderBase.java:738-789) is decoded up front
 * on the GPU; each page then gets a GpuValuesReader over its slice of the dense column.
 */
package org.apache.parquet.column.values.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import org.apache.parquet.io.ParquetDecodingException;

public final class GpuPageBatch {
  final byte[] pageDescs;
  final int[] pageCounts;
  final Object[] values;
  final byte[][] defLevels;
  final byte[][] repLevels;
  final byte[][] binary;
  final int[] physicalType;
  final int[] typeLength;
  final int[] flags;
  final int code;
  final int errorPage;
  final long errorIndex;
  final int errorKind;
  final long[] valuesWritten;
  /** Per page: its column, and the index of its first value in that column's dense output. */
  private final int[] pageColumn;
  private final long[] pageFirst;

  /**
   * @param pageBytes direct or heap buffer; [position, limit) holds every page body (and dictionary
   *     page) the descriptors refer to (descriptor offsets are relative to position)
   * @param pageDescs packed pqg_page_desc[] (PqGpu.frameChunk output, concatenated per chunk)
   * @param columnDescs packed pqg_column_desc[] without output pointers
   */
  public GpuPageBatch(long ctx, ByteBuffer pageBytes, byte[] pageDescs, byte[] columnDescs, Object[] values,
      byte[][] defLevels, byte[][] repLevels, byte[][] binary) {
    int nPages = pageDescs.length / PqGpu.PAGE_DESC_BYTES;
    int nCols = columnDescs.length / PqGpu.COLUMN_DESC_BYTES;
    this.pageDescs = pageDescs;
    this.pageCounts = new int[nPages];
    this.values = values;
    this.defLevels = defLevels;
    this.repLevels = repLevels;
    this.binary = binary;
    ByteBuffer cd = ByteBuffer.wrap(columnDescs).order(ByteOrder.LITTLE_ENDIAN);
    physicalType = new int[nCols];
    typeLength = new int[nCols];
    flags = new int[nCols];
    for (int i = 0; i < nCols; i++) {
      int b = i * PqGpu.COLUMN_DESC_BYTES;
      physicalType[i] = cd.getInt(b);
      typeLength[i] = cd.getInt(b + 4);
      flags[i] = cd.getInt(b + 36);
    }
    long[] r = PqGpu.decodeHost(ctx, pageBytes, pageDescs, columnDescs, values, defLevels, repLevels, binary, pageCounts);
    code = (int) r[0];
    errorPage = (int) r[1];
    errorIndex = r[2];
    errorKind = (int) r[3];
    valuesWritten = new long[nCols];
    System.arraycopy(r, 4, valuesWritten, 0, nCols);
    // one pass: each page's column and its first value (prefix sum of the value counts per column)
    ByteBuffer pd = ByteBuffer.wrap(pageDescs).order(ByteOrder.LITTLE_ENDIAN);
    pageColumn = new int[nPages];
    pageFirst = new long[nPages];
    long[] acc = new long[Math.max(nCols, 1)];
    for (int p = 0; p < nPages; p++) {
      int c = pd.getInt(p * PqGpu.PAGE_DESC_BYTES + 16);
      pageColumn[p] = c;
      if (c >= 0 && c < nCols) {
        pageFirst[p] = acc[c];
        acc[c] += pageCounts[p];
      }
    }
  }

  public int pageCount() {
    return pageColumn.length;
  }

  /** The reader of one data page (the ValuesReader ColumnReaderBase.initDataReader would create). O(1). */
  public GpuValuesReader reader(int page) {
    int column = pageColumn[page];
    long first = pageFirst[page];
    long errorAt = -1;
    if (code != 0) {
      if (errorPage < 0 || page > errorPage || (page == errorPage && errorKind == 2)) {
        throw exception(code, "page " + page + " of the batch cannot be read (batch failed at page " + errorPage + ")");
      }
      if (page == errorPage) errorAt = first + errorIndex;
    }
    return new GpuValuesReader(this, column, first, first + pageCounts[page], errorAt);
  }

  RuntimeException exception(int c, String what) {
    String cls = PqGpu.exceptionClass(c);
    String msg = what + " (pqg error " + c + ")";
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

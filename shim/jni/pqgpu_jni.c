/*
 * pqgpu_jni.c — JNI glue of org.apache.parquet.column.values.gpu.PqGpu (shim/java/) over the C ABI
 * of libpqgpu.so (include/pqgpu.h, include/pqgpu_reader.h). Build where a JDK exists:
 *   make -C shim JAVA_HOME=/path/to/jdk        (-> shim/libpqgpu_jni.so, links libpqgpu.so)
 * The build image has no JDK; every C entry this file calls is exercised from C by
 * tests/c/harness.c (tests/test_c_harness.py) with the same call sequence.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "pqgpu.h"
#include "pqgpu_reader.h"

static void throw_code(JNIEnv* env, int code, const char* msg) {
  const char* cls = pqg_java_exception(code);
  jclass c = (*env)->FindClass(env, cls ? cls : "java/lang/IllegalStateException");
  if (c) (*env)->ThrowNew(env, c, msg);
}

JNIEXPORT jint JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_deviceCount(JNIEnv* env, jclass k) {
  (void)env;
  (void)k;
  return pqg_device_count();
}

JNIEXPORT jlong JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_ctxCreate(JNIEnv* env, jclass k, jint dev) {
  (void)k;
  pqg_ctx* ctx = NULL;
  int rc = pqg_ctx_create(dev, NULL, &ctx);
  if (rc) {
    throw_code(env, rc, "pqg_ctx_create failed");
    return 0;
  }
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_ctxDestroy(JNIEnv* env, jclass k, jlong ctx) {
  (void)env;
  (void)k;
  pqg_ctx_destroy((pqg_ctx*)(intptr_t)ctx);
}

JNIEXPORT jstring JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_exceptionClass(JNIEnv* env, jclass k,
                                                                                        jint code) {
  (void)k;
  const char* c = pqg_java_exception(code);
  return c ? (*env)->NewStringUTF(env, c) : NULL;
}

/* Input bytes of a host-only call: a direct buffer's address, or a byte[] pinned for its duration.
 * [offset, offset + length) is what the Java side passes (the buffer's position() .. limit()). */
typedef struct {
  jbyteArray array;
  const uint8_t* base;
  void* pinned;
} in_bytes;

static int in_check(JNIEnv* env, jobject direct, jbyteArray array, jint offset, jint length, const char* what) {
  jlong cap = direct ? (*env)->GetDirectBufferCapacity(env, direct) : array ? (*env)->GetArrayLength(env, array) : -1;
  if ((direct && !(*env)->GetDirectBufferAddress(env, direct)) || cap < 0 || offset < 0 || length < 0 ||
      (jlong)offset + length > cap) {
    throw_code(env, PQG_ERR_INVALID_ARG, what);
    return 0;
  }
  return 1;
}

/* Pin (array) or address (direct) the input; no other JNI call may follow until in_release. Used
 * only around host-side parsing (pqg_frame_chunk: no device call, no waiting). */
static const uint8_t* in_acquire(JNIEnv* env, jobject direct, jbyteArray array, jint offset, in_bytes* ib) {
  ib->array = array;
  ib->pinned = NULL;
  if (direct) {
    ib->base = (const uint8_t*)(*env)->GetDirectBufferAddress(env, direct);
  } else {
    ib->pinned = (*env)->GetPrimitiveArrayCritical(env, array, NULL);
    ib->base = (const uint8_t*)ib->pinned;
  }
  return ib->base ? ib->base + offset : NULL;
}

static void in_release(JNIEnv* env, in_bytes* ib) {
  if (ib->pinned) (*env)->ReleasePrimitiveArrayCritical(env, ib->array, ib->pinned, JNI_ABORT);
  ib->pinned = NULL;
}

static jbyteArray frame_chunk(JNIEnv* env, jobject direct, jbyteArray array, jint offset, jint length,
                              jlong value_count, jboolean verify_crc, jint codec, jlong chunk_offset, jint column,
                              jlongArray dict_info) {
  if (!in_check(env, direct, array, offset, length, "frameChunk: bad buffer range")) return NULL;
  if (!dict_info || (*env)->GetArrayLength(env, dict_info) < 4) {
    throw_code(env, PQG_ERR_INVALID_ARG, "frameChunk: dictInfo needs 4 entries");
    return NULL;
  }
  pqg_status st;
  int n_hdr = 0, cap = 64;
  pqg_page_header* hdr = NULL;
  int rc;
  for (;;) { /* grow to the header count the library reports */
    free(hdr);
    hdr = (pqg_page_header*)calloc((size_t)cap, sizeof(*hdr));
    if (!hdr) {
      throw_code(env, PQG_ERR_INVALID_ARG, "out of memory");
      return NULL;
    }
    in_bytes ib;
    const uint8_t* bytes = in_acquire(env, direct, array, offset, &ib);
    rc = bytes ? pqg_frame_chunk(bytes, (uint64_t)length, value_count, verify_crc ? 1 : 0, hdr, cap, &n_hdr, &st)
               : PQG_ERR_INVALID_ARG;
    in_release(env, &ib);
    if (rc == PQG_ERR_INVALID_ARG && n_hdr > cap) {
      cap = n_hdr;
      continue;
    }
    break;
  }
  if (rc) {
    free(hdr);
    throw_code(env, rc, st.message);
    return NULL;
  }
  pqg_column_desc col;
  memset(&col, 0, sizeof(col));
  col.dict_offset = -1;
  pqg_page_desc* pages = (pqg_page_desc*)calloc((size_t)n_hdr + 1, sizeof(*pages));
  int n_pages = 0;
  rc = pages ? pqg_pages_from_headers(hdr, n_hdr, codec, (uint64_t)chunk_offset, column, &col, pages, n_hdr + 1,
                                      &n_pages, &st)
             : PQG_ERR_INVALID_ARG;
  free(hdr);
  if (rc) {
    free(pages);
    throw_code(env, rc, pages ? st.message : "out of memory");
    return NULL;
  }
  jlong info[4] = {col.dict_offset, col.dict_size, col.dict_num_values, col.dict_encoding};
  (*env)->SetLongArrayRegion(env, dict_info, 0, 4, info);
  jbyteArray out = (*env)->NewByteArray(env, (jsize)(n_pages * (int)sizeof(pqg_page_desc)));
  if (out) (*env)->SetByteArrayRegion(env, out, 0, (jsize)(n_pages * (int)sizeof(pqg_page_desc)), (const jbyte*)pages);
  free(pages);
  return out;
}

JNIEXPORT jbyteArray JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_frameChunkDirect(
    JNIEnv* env, jclass k, jobject chunk, jint offset, jint length, jlong value_count, jboolean verify_crc, jint codec,
    jlong chunk_offset, jint column, jlongArray dict_info) {
  (void)k;
  return frame_chunk(env, chunk, NULL, offset, length, value_count, verify_crc, codec, chunk_offset, column, dict_info);
}

JNIEXPORT jbyteArray JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_frameChunkArray(
    JNIEnv* env, jclass k, jbyteArray chunk, jint offset, jint length, jlong value_count, jboolean verify_crc,
    jint codec, jlong chunk_offset, jint column, jlongArray dict_info) {
  (void)k;
  return frame_chunk(env, NULL, chunk, offset, length, value_count, verify_crc, codec, chunk_offset, column, dict_info);
}

/* Copy the input bytes (direct buffer address or a heap array region) into `dst` without holding
 * the array: GetByteArrayRegion copies, no critical region. */
static int copy_in(JNIEnv* env, jobject direct, jbyteArray array, jint offset, jint length, uint8_t* dst) {
  if (length == 0) return 1;
  if (direct) {
    const uint8_t* base = (const uint8_t*)(*env)->GetDirectBufferAddress(env, direct);
    if (!base) return 0;
    memcpy(dst, base + offset, (size_t)length);
    return 1;
  }
  (*env)->GetByteArrayRegion(env, array, offset, length, (jbyte*)dst);
  return !(*env)->ExceptionCheck(env);
}

/* `arrays[i]` as a primitive array of at least `n` elements of `kind` ('J' long, 'I' int, 'F' float,
 * 'D' double, 'B' byte): the caller's array when it is long enough, else a new one of exactly n
 * stored back into arrays[i]. NULL with an exception pending on failure. */
static jarray out_array(JNIEnv* env, jobjectArray arrays, jsize i, char kind, jsize n) {
  jarray a = (jarray)(*env)->GetObjectArrayElement(env, arrays, i);
  if (a) {
    const char* sig = kind == 'J' ? "[J" : kind == 'I' ? "[I" : kind == 'F' ? "[F" : kind == 'D' ? "[D" : "[B";
    jclass want = (*env)->FindClass(env, sig);
    if (!want) return NULL;
    const jboolean ok = (*env)->IsInstanceOf(env, a, want);
    (*env)->DeleteLocalRef(env, want);
    if (!ok) {
      (*env)->DeleteLocalRef(env, a);
      throw_code(env, PQG_ERR_INVALID_ARG, "decodeHost: an output array has the wrong element type");
      return NULL;
    }
    if ((*env)->GetArrayLength(env, a) >= n) return a;
    (*env)->DeleteLocalRef(env, a);
  }
  switch (kind) {
    case 'J': a = (*env)->NewLongArray(env, n); break;
    case 'I': a = (*env)->NewIntArray(env, n); break;
    case 'F': a = (*env)->NewFloatArray(env, n); break;
    case 'D': a = (*env)->NewDoubleArray(env, n); break;
    default: a = (*env)->NewByteArray(env, n); break;
  }
  if (a) (*env)->SetObjectArrayElement(env, arrays, i, a);
  return a;
}

/* Copy `bytes` bytes of pinned library memory into a Java array: a critical region around a plain
 * (multi-threaded) memcpy only — no JNI call, no device call, no waiting inside it. */
static void copy_out(JNIEnv* env, jarray a, const void* src, uint64_t bytes) {
  if (!bytes) return;
  void* dst = (*env)->GetPrimitiveArrayCritical(env, a, NULL);
  if (!dst) return; /* OutOfMemoryError pending */
  pqg_copy_out(dst, src, bytes);
  (*env)->ReleasePrimitiveArrayCritical(env, a, dst, 0);
}

/* Decode a batch through the staged path: the page bytes are copied into the library's pinned input
 * (no Java array is held while the device works), decoded, and each output is copied from the
 * library's pinned output into its Java array afterwards. */
static jlongArray decode_host(JNIEnv* env, jlong ctx, jobject direct, jbyteArray array, jint offset, jint length,
                              jbyteArray page_descs, jbyteArray column_descs, jobjectArray values,
                              jobjectArray def_levels, jobjectArray rep_levels, jobjectArray binary,
                              jintArray page_counts) {
  if (!in_check(env, direct, array, offset, length, "decodeHost: bad buffer range")) return NULL;
  const jsize n_pages = (*env)->GetArrayLength(env, page_descs) / (jsize)sizeof(pqg_page_desc);
  const jsize n_cols = (*env)->GetArrayLength(env, column_descs) / (jsize)sizeof(pqg_column_desc);
  if ((*env)->GetArrayLength(env, page_counts) < n_pages || (*env)->GetArrayLength(env, values) < n_cols ||
      (*env)->GetArrayLength(env, def_levels) < n_cols || (*env)->GetArrayLength(env, rep_levels) < n_cols ||
      (*env)->GetArrayLength(env, binary) < n_cols) {
    throw_code(env, PQG_ERR_INVALID_ARG, "decodeHost: array arguments shorter than the descriptors");
    return NULL;
  }
  pqg_page_desc* pd = (pqg_page_desc*)malloc(sizeof(pqg_page_desc) * (size_t)(n_pages + 1));
  pqg_column_desc* cd = (pqg_column_desc*)malloc(sizeof(pqg_column_desc) * (size_t)(n_cols + 1));
  uint32_t* counts = (uint32_t*)calloc((size_t)n_pages + 1, sizeof(uint32_t));
  pqg_page_error* pe = (pqg_page_error*)calloc((size_t)n_pages + 1, sizeof(pqg_page_error));
  const jsize n_res = 4 + n_cols + 3 * n_pages;
  jlong* res = (jlong*)calloc((size_t)n_res, sizeof(jlong));
  jlongArray out = NULL;
  if (!pd || !cd || !counts || !pe || !res) {
    throw_code(env, PQG_ERR_INVALID_ARG, "out of memory");
    goto done;
  }
  (*env)->GetByteArrayRegion(env, page_descs, 0, n_pages * (jsize)sizeof(pqg_page_desc), (jbyte*)pd);
  (*env)->GetByteArrayRegion(env, column_descs, 0, n_cols * (jsize)sizeof(pqg_column_desc), (jbyte*)cd);
  pqg_ctx* c = (pqg_ctx*)(intptr_t)ctx;
  uint8_t* in = NULL;
  pqg_status st;
  memset(&st, 0, sizeof(st));
  int rc = pqg_host_input(c, (uint64_t)length, &in);
  if (rc) {
    throw_code(env, rc, "pqg_host_input failed");
    goto done;
  }
  if (!copy_in(env, direct, array, offset, length, in)) goto done;
  rc = pqg_decode_staged(c, (uint64_t)length, cd, n_cols, pd, n_pages, counts, &st);
  if (rc == PQG_ERR_HIP || rc == PQG_ERR_NO_DEVICE || rc == PQG_ERR_TIMEOUT || (rc == PQG_ERR_INVALID_ARG && st.page == -1)) {
    throw_code(env, rc, st.message); /* the backend failed or the call was malformed: not a decode error */
    goto done;
  }
  if (rc && pqg_page_errors(c, pe, n_pages) != PQG_OK) {
    /* no plan was made (a descriptor refused before the launch): the call's own status is the error */
    throw_code(env, rc, st.message);
    goto done;
  }
  for (jsize i = 0; i < n_cols; i++) {
    pqg_staged_output o;
    if (pqg_staged_column(c, i, &o) != PQG_OK) {
      throw_code(env, PQG_ERR_INVALID_ARG, "pqg_staged_column failed");
      goto done;
    }
    const int ids = (cd[i].flags & PQG_COLUMN_DICTIONARY_IDS) != 0;
    const int t = cd[i].physical_type;
    char kind = 'B';
    uint64_t n = o.n_values, w = 1;
    if (ids) { kind = 'I'; w = 4; }
    else if (t == PQG_INT32) { kind = 'I'; w = 4; }
    else if (t == PQG_INT64) { kind = 'J'; w = 8; }
    else if (t == PQG_FLOAT) { kind = 'F'; w = 4; }
    else if (t == PQG_DOUBLE) { kind = 'D'; w = 8; }
    else if (t == PQG_BYTE_ARRAY) { kind = 'J'; w = 8; n = o.n_values + 1; }  /* offsets[n + 1] */
    else if (t == PQG_INT96) { n = o.n_values * 12; }
    else if (t == PQG_FIXED_LEN_BYTE_ARRAY) { n = o.n_values * (uint64_t)cd[i].type_length; }
    if (n > 0x7fffffffull || o.n_slots > 0x7fffffffull || o.n_binary > 0x7fffffffull) {
      throw_code(env, PQG_ERR_INVALID_ARG, "decodeHost: a column exceeds a Java array");
      goto done;
    }
    jarray a = out_array(env, values, i, kind, (jsize)n);
    if (!a) goto done;
    copy_out(env, a, o.values, n * w);
    (*env)->DeleteLocalRef(env, a);
    if (o.def_levels) {
      if (!(a = out_array(env, def_levels, i, 'B', (jsize)o.n_slots))) goto done;
      copy_out(env, a, o.def_levels, o.n_slots);
      (*env)->DeleteLocalRef(env, a);
    }
    if (o.rep_levels) {
      if (!(a = out_array(env, rep_levels, i, 'B', (jsize)o.n_slots))) goto done;
      copy_out(env, a, o.rep_levels, o.n_slots);
      (*env)->DeleteLocalRef(env, a);
    }
    if (o.binary) {
      if (!(a = out_array(env, binary, i, 'B', (jsize)o.n_binary))) goto done;
      copy_out(env, a, o.binary, o.n_binary);
      (*env)->DeleteLocalRef(env, a);
    }
    res[4 + i] = (jlong)o.n_values;
    if ((*env)->ExceptionCheck(env)) goto done;
  }
  (*env)->SetIntArrayRegion(env, page_counts, 0, n_pages, (const jint*)counts);
  /* {code, page, value_index, 0, values_written[n_cols], (code, phase, index) per page} */
  res[0] = rc;
  res[1] = rc ? st.page : -1;
  res[2] = rc ? st.value_index : -1;
  for (jsize p = 0; p < n_pages; p++) {
    res[4 + n_cols + 3 * p] = pe[p].code;
    res[4 + n_cols + 3 * p + 1] = pe[p].phase;
    res[4 + n_cols + 3 * p + 2] = pe[p].index;
  }
  out = (*env)->NewLongArray(env, n_res);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, n_res, res);
done:
  free(res); free(pd); free(cd); free(counts); free(pe);
  return out;
}

JNIEXPORT jlongArray JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_decodeHostDirect(
    JNIEnv* env, jclass k, jlong ctx, jobject page_bytes, jint offset, jint length, jbyteArray page_descs,
    jbyteArray column_descs, jobjectArray values, jobjectArray def_levels, jobjectArray rep_levels,
    jobjectArray binary, jintArray page_counts) {
  (void)k;
  return decode_host(env, ctx, page_bytes, NULL, offset, length, page_descs, column_descs, values, def_levels,
                     rep_levels, binary, page_counts);
}

JNIEXPORT jlongArray JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_decodeHostArray(
    JNIEnv* env, jclass k, jlong ctx, jbyteArray page_bytes, jint offset, jint length, jbyteArray page_descs,
    jbyteArray column_descs, jobjectArray values, jobjectArray def_levels, jobjectArray rep_levels,
    jobjectArray binary, jintArray page_counts) {
  (void)k;
  return decode_host(env, ctx, NULL, page_bytes, offset, length, page_descs, column_descs, values, def_levels,
                     rep_levels, binary, page_counts);
}

static void throw_router(JNIEnv* env, int rc, const char* what) {
  /* SingleBufferInputStream.slice past the end: EOFException; the router declares IOException */
  if (rc == PQG_ERR_EOF) {
    jclass c = (*env)->FindClass(env, "java/io/EOFException");
    if (c) (*env)->ThrowNew(env, c, "routerRead: input shorter than count * bitWidth / 8 bytes");
  } else if (rc > 0) {
    throw_code(env, rc, what);
  }
}

/* Router reads copy their input in (GetByteArrayRegion / direct address) and their output out
 * (SetIntArrayRegion): no Java array is held while the device works. */
static void router_runs(JNIEnv* env, jlong ctx, jint bit_width, jobject direct, jbyteArray array, jint offset,
                        jint length, const uint64_t* offs, const uint32_t* counts, jint n_runs, jintArray out) {
  uint64_t total = 0;
  for (jint r = 0; r < n_runs; r++) total += counts[r];
  if ((*env)->GetArrayLength(env, out) < (jlong)total) {
    throw_code(env, PQG_ERR_INVALID_ARG, "routerRead: output array too short");
    return;
  }
  uint8_t* in = (uint8_t*)malloc((size_t)length + 1);
  int32_t* dst = (int32_t*)malloc(4 * (size_t)total + 4);
  int rc = in && dst ? PQG_OK : PQG_ERR_INVALID_ARG;
  if (!rc && !copy_in(env, direct, array, offset, length, in)) rc = -1; /* exception pending */
  if (!rc) rc = pqg_router_read_runs((pqg_ctx*)(intptr_t)ctx, bit_width, in, (size_t)length, offs, counts, n_runs, dst);
  if (!rc && total) (*env)->SetIntArrayRegion(env, out, 0, (jsize)total, (const jint*)dst);
  free(in);
  free(dst);
  throw_router(env, rc, "pqg_router_read_runs failed");
}

static void router_read(JNIEnv* env, jlong ctx, jint bit_width, jobject direct, jbyteArray array, jint offset,
                        jint length, jint count, jintArray out) {
  if (!in_check(env, direct, array, offset, length, "routerRead: bad buffer range")) return;
  if (count < 0) {
    throw_code(env, PQG_ERR_INVALID_ARG, "routerRead arguments");
    return;
  }
  const uint64_t off0 = 0;
  const uint32_t cnt = (uint32_t)count;
  router_runs(env, ctx, bit_width, direct, array, offset, length, &off0, &cnt, 1, out);
}

static void router_read_batch(JNIEnv* env, jlong ctx, jint bit_width, jobject direct, jbyteArray array, jint offset,
                              jint length, jlongArray run_offsets, jintArray run_counts, jint n_runs, jintArray out) {
  if (!in_check(env, direct, array, offset, length, "routerReadBatch: bad buffer range")) return;
  if (n_runs < 0 || (*env)->GetArrayLength(env, run_offsets) < n_runs ||
      (*env)->GetArrayLength(env, run_counts) < n_runs) {
    throw_code(env, PQG_ERR_INVALID_ARG, "routerReadBatch arguments");
    return;
  }
  uint64_t* offs = (uint64_t*)malloc(8 * (size_t)n_runs + 8);
  uint32_t* counts = (uint32_t*)malloc(4 * (size_t)n_runs + 4);
  if (offs && counts) {
    (*env)->GetLongArrayRegion(env, run_offsets, 0, n_runs, (jlong*)offs);
    (*env)->GetIntArrayRegion(env, run_counts, 0, n_runs, (jint*)counts);
    int bad = 0;
    for (jint r = 0; r < n_runs; r++) bad |= (int64_t)offs[r] < 0 || (int32_t)counts[r] < 0;
    if (bad) throw_code(env, PQG_ERR_INVALID_ARG, "routerReadBatch: negative offset or count");
    else router_runs(env, ctx, bit_width, direct, array, offset, length, offs, counts, n_runs, out);
  } else {
    throw_code(env, PQG_ERR_INVALID_ARG, "out of memory");
  }
  free(offs);
  free(counts);
}

/* ParquetReadRouter.read with the contract kept (values in `out` on return), one device round trip per
 * page (pqg_router_read_page). [offset, offset + length) is the caller's stream from the run's data start
 * to its end. A direct buffer is read in place; a heap array is probed with the run's bytes only
 * (pqg_router_cache_lookup: a host-only copy of count * bitWidth / 8 bytes) and copied whole only on a
 * miss. No Java array is held while the device works. */
static void router_page(JNIEnv* env, jlong ctx, jint bit_width, jobject direct, jbyteArray array, jint offset,
                        jint length, jint count, jintArray out) {
  if (!in_check(env, direct, array, offset, length, "routerReadPage: bad buffer range")) return;
  if (count < 0 || bit_width < 0 || bit_width > 32 || (*env)->GetArrayLength(env, out) < count) {
    throw_code(env, PQG_ERR_INVALID_ARG, "routerReadPage arguments");
    return;
  }
  pqg_ctx* c = (pqg_ctx*)(intptr_t)ctx;
  const uint64_t need = (uint64_t)count * (uint64_t)bit_width / 8u;
  int32_t* dst = (int32_t*)malloc(4 * (size_t)count + 4);
  int rc = dst ? PQG_OK : PQG_ERR_INVALID_ARG;
  if (!rc && direct) {
    const uint8_t* base = (const uint8_t*)(*env)->GetDirectBufferAddress(env, direct);
    rc = pqg_router_read_page(c, bit_width, base + offset, (size_t)length, count, dst);
  } else if (!rc) {
    int hit = 0;
    if (need <= (uint64_t)length) {
      uint8_t* run = (uint8_t*)malloc((size_t)need + 1);
      rc = run ? PQG_OK : PQG_ERR_INVALID_ARG;
      if (!rc && !copy_in(env, NULL, array, offset, (jint)need, run)) rc = -1; /* exception pending */
      if (!rc) rc = pqg_router_cache_lookup(c, bit_width, run, (size_t)length, count, dst, &hit);
      free(run);
    }
    if (!rc && !hit) {
      uint8_t* tail = (uint8_t*)malloc((size_t)length + 1);
      rc = tail ? PQG_OK : PQG_ERR_INVALID_ARG;
      if (!rc && !copy_in(env, NULL, array, offset, length, tail)) rc = -1;
      if (!rc) rc = pqg_router_read_page(c, bit_width, tail, (size_t)length, count, dst);
      free(tail);
    }
  }
  if (!rc && count) (*env)->SetIntArrayRegion(env, out, 0, count, (const jint*)dst);
  free(dst);
  throw_router(env, rc, "pqg_router_read_page failed");
}

JNIEXPORT void JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_routerReadPageDirect(
    JNIEnv* env, jclass k, jlong ctx, jint bit_width, jobject in, jint offset, jint length, jint count, jintArray out) {
  (void)k;
  router_page(env, ctx, bit_width, in, NULL, offset, length, count, out);
}

JNIEXPORT void JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_routerReadPageArray(
    JNIEnv* env, jclass k, jlong ctx, jint bit_width, jbyteArray in, jint offset, jint length, jint count,
    jintArray out) {
  (void)k;
  router_page(env, ctx, bit_width, NULL, in, offset, length, count, out);
}

JNIEXPORT void JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_routerReadBatchDirect(
    JNIEnv* env, jclass k, jlong ctx, jint bit_width, jobject in, jint offset, jint length, jlongArray run_offsets,
    jintArray run_counts, jint n_runs, jintArray out) {
  (void)k;
  router_read_batch(env, ctx, bit_width, in, NULL, offset, length, run_offsets, run_counts, n_runs, out);
}

JNIEXPORT void JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_routerReadBatchArray(
    JNIEnv* env, jclass k, jlong ctx, jint bit_width, jbyteArray in, jint offset, jint length, jlongArray run_offsets,
    jintArray run_counts, jint n_runs, jintArray out) {
  (void)k;
  router_read_batch(env, ctx, bit_width, NULL, in, offset, length, run_offsets, run_counts, n_runs, out);
}

JNIEXPORT void JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_routerReadDirect(
    JNIEnv* env, jclass k, jlong ctx, jint bit_width, jobject in, jint offset, jint length, jint count, jintArray out) {
  (void)k;
  router_read(env, ctx, bit_width, in, NULL, offset, length, count, out);
}

JNIEXPORT void JNICALL Java_org_apache_parquet_column_values_gpu_PqGpu_routerReadArray(
    JNIEnv* env, jclass k, jlong ctx, jint bit_width, jbyteArray in, jint offset, jint length, jint count,
    jintArray out) {
  (void)k;
  router_read(env, ctx, bit_width, NULL, in, offset, length, count, out);
}

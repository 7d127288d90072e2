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

/* Input bytes of a call: a direct buffer's address, or a byte[] pinned for the call's duration.
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

/* Pin (array) or address (direct) the input; no other JNI call may follow until in_release. */
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

/* The output arrays (and a heap input array) stay pinned (GetPrimitiveArrayCritical) for the one
 * pqg_decode_host call: it stages the input into pinned host memory and copies the decoded values
 * straight into the outputs; no JNI call is made while they are pinned. */
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
  if ((*env)->EnsureLocalCapacity(env, n_cols * 4 + 16) != 0) return NULL; /* OutOfMemoryError pending */
  pqg_page_desc* pd = (pqg_page_desc*)malloc(sizeof(pqg_page_desc) * (size_t)(n_pages + 1));
  pqg_column_desc* cd = (pqg_column_desc*)malloc(sizeof(pqg_column_desc) * (size_t)(n_cols + 1));
  uint32_t* counts = (uint32_t*)calloc((size_t)n_pages + 1, sizeof(uint32_t));
  jobject* pinned = (jobject*)calloc((size_t)n_cols * 4 + 1, sizeof(jobject));
  void** ptrs = (void**)calloc((size_t)n_cols * 4 + 1, sizeof(void*));
  jlong* res = (jlong*)calloc((size_t)n_cols + 4, sizeof(jlong));
  if (!pd || !cd || !counts || !pinned || !ptrs || !res) {
    free(pd); free(cd); free(counts); free(pinned); free(ptrs); free(res);
    throw_code(env, PQG_ERR_INVALID_ARG, "out of memory");
    return NULL;
  }
  (*env)->GetByteArrayRegion(env, page_descs, 0, n_pages * (jsize)sizeof(pqg_page_desc), (jbyte*)pd);
  (*env)->GetByteArrayRegion(env, column_descs, 0, n_cols * (jsize)sizeof(pqg_column_desc), (jbyte*)cd);
  /* element counts first (GetArrayLength is not allowed inside a critical region) */
  for (jsize i = 0; i < n_cols; i++) {
    jobject arrs[4] = {(*env)->GetObjectArrayElement(env, values, i), (*env)->GetObjectArrayElement(env, def_levels, i),
                       (*env)->GetObjectArrayElement(env, rep_levels, i), (*env)->GetObjectArrayElement(env, binary, i)};
    for (int a = 0; a < 4; a++) pinned[4 * i + a] = arrs[a];
    const jsize nv = arrs[0] ? (*env)->GetArrayLength(env, (jarray)arrs[0]) : 0;
    const jsize nd = arrs[1] ? (*env)->GetArrayLength(env, (jarray)arrs[1]) : 0;
    const jsize nr = arrs[2] ? (*env)->GetArrayLength(env, (jarray)arrs[2]) : 0;
    const jsize nb = arrs[3] ? (*env)->GetArrayLength(env, (jarray)arrs[3]) : 0;
    /* capacity in elements of the output: an ids column's int[] holds one uint32 id per value
     * whatever the physical type; only the byte[] of FIXED_LEN_BYTE_ARRAY / INT96 values holds
     * type-length bytes per value */
    const int ids = (cd[i].flags & PQG_COLUMN_DICTIONARY_IDS) != 0;
    const int fixed_bytes = !ids && (cd[i].physical_type == PQG_FIXED_LEN_BYTE_ARRAY || cd[i].physical_type == PQG_INT96);
    const int w = cd[i].physical_type == PQG_INT96 ? 12 : cd[i].type_length;
    cd[i].values_capacity = fixed_bytes ? (w > 0 ? (uint64_t)nv / (uint64_t)w : 0) : (uint64_t)nv;
    cd[i].levels_capacity = (uint64_t)(nd > nr ? nd : nr);
    cd[i].binary_capacity = (uint64_t)nb;
  }
  for (jsize j = 0; j < n_cols * 4; j++)
    ptrs[j] = pinned[j] ? (*env)->GetPrimitiveArrayCritical(env, (jarray)pinned[j], NULL) : NULL;
  for (jsize i = 0; i < n_cols; i++) {
    cd[i].values = ptrs[4 * i];
    cd[i].def_levels = (uint8_t*)ptrs[4 * i + 1];
    cd[i].rep_levels = (uint8_t*)ptrs[4 * i + 2];
    cd[i].binary_data = (uint8_t*)ptrs[4 * i + 3];
  }
  pqg_status st;
  memset(&st, 0, sizeof(st));
  in_bytes ib;
  const uint8_t* bytes = in_acquire(env, direct, array, offset, &ib);
  const int rc = bytes ? pqg_decode_host((pqg_ctx*)(intptr_t)ctx, bytes, (uint64_t)length, cd, n_cols, pd, n_pages,
                                         counts, &st)
                       : PQG_ERR_INVALID_ARG;
  in_release(env, &ib);
  for (jsize j = n_cols * 4 - 1; j >= 0; j--)
    if (ptrs[j]) (*env)->ReleasePrimitiveArrayCritical(env, (jarray)pinned[j], ptrs[j], 0);
  (*env)->SetIntArrayRegion(env, page_counts, 0, n_pages, (const jint*)counts);
  /* {code, page, value_index, kind, values_written...}: kind 1 = a value error raised lazily at its
   * read, 2 = a page error raised at initFromPage (pqg_vr_init_from_page's rule) */
  res[0] = rc;
  res[1] = rc ? st.page : -1;
  res[2] = rc ? st.value_index : -1;
  res[3] = rc == 0 ? 0 : strncmp(st.message, "value decode", 12) == 0 ? 1 : 2;
  for (jsize i = 0; i < n_cols; i++) res[4 + i] = (jlong)cd[i].values_written;
  jlongArray out = (*env)->NewLongArray(env, n_cols + 4);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, n_cols + 4, res);
  if (rc == PQG_ERR_INVALID_ARG && st.page == -1) throw_code(env, rc, st.message); /* capacity: API misuse */
  else if (rc == PQG_ERR_HIP || rc == PQG_ERR_NO_DEVICE || rc == PQG_ERR_TIMEOUT) throw_code(env, rc, st.message);
  free(res); free(pd); free(cd); free(counts); free(pinned); free(ptrs);
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

static void router_read(JNIEnv* env, jlong ctx, jint bit_width, jobject direct, jbyteArray array, jint offset,
                        jint length, jint count, jintArray out) {
  if (!in_check(env, direct, array, offset, length, "routerRead: bad buffer range")) return;
  if (count < 0 || (*env)->GetArrayLength(env, out) < count) {
    throw_code(env, PQG_ERR_INVALID_ARG, "routerRead arguments");
    return;
  }
  int32_t* dst = (int32_t*)(*env)->GetPrimitiveArrayCritical(env, out, NULL);
  in_bytes ib;
  const uint8_t* bytes = dst ? in_acquire(env, direct, array, offset, &ib) : NULL;
  const int rc = bytes ? pqg_router_read((pqg_ctx*)(intptr_t)ctx, bit_width, bytes, (size_t)length, count, dst)
                       : PQG_ERR_INVALID_ARG;
  if (dst) {
    in_release(env, &ib);
    (*env)->ReleasePrimitiveArrayCritical(env, out, dst, 0);
  }
  /* SingleBufferInputStream.slice past the end: EOFException; the router declares IOException */
  if (rc == PQG_ERR_EOF) {
    jclass c = (*env)->FindClass(env, "java/io/EOFException");
    if (c) (*env)->ThrowNew(env, c, "routerRead: input shorter than count * bitWidth / 8 bytes");
  } else if (rc) {
    throw_code(env, rc, "pqg_router_read failed");
  }
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

/*
 * jni.h stand-in for a COMPILE CHECK ONLY of shim/jni/pqgpu_jni.c (tests/test_abi.py): the build
 * image has no JDK. It declares the JNI types and, in a struct of the same shape as the C form of
 * JNIEnv, exactly the functions the glue calls, with their signatures from the JNI specification.
 * Nothing is linked or run against it; the real header comes with the JDK (make -C shim).
 */
#ifndef PQG_JNI_STUB_H
#define PQG_JNI_STUB_H
#include <stdint.h>

typedef uint8_t jboolean;
typedef int8_t jbyte;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef int32_t jint;
typedef int64_t jlong;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jfloatArray;
typedef jarray jdoubleArray;

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_ABORT 2

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv*, const char*);
  jint (*ThrowNew)(JNIEnv*, jclass, const char*);
  jboolean (*ExceptionCheck)(JNIEnv*);
  void (*DeleteLocalRef)(JNIEnv*, jobject);
  jboolean (*IsInstanceOf)(JNIEnv*, jobject, jclass);
  jstring (*NewStringUTF)(JNIEnv*, const char*);
  jsize (*GetArrayLength)(JNIEnv*, jarray);
  jobject (*GetObjectArrayElement)(JNIEnv*, jobjectArray, jsize);
  void (*SetObjectArrayElement)(JNIEnv*, jobjectArray, jsize, jobject);
  jbyteArray (*NewByteArray)(JNIEnv*, jsize);
  jintArray (*NewIntArray)(JNIEnv*, jsize);
  jlongArray (*NewLongArray)(JNIEnv*, jsize);
  jfloatArray (*NewFloatArray)(JNIEnv*, jsize);
  jdoubleArray (*NewDoubleArray)(JNIEnv*, jsize);
  void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);
  void (*GetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, jint*);
  void (*GetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, jlong*);
  void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);
  void (*SetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, const jint*);
  void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
  void* (*GetPrimitiveArrayCritical)(JNIEnv*, jarray, jboolean*);
  void (*ReleasePrimitiveArrayCritical)(JNIEnv*, jarray, void*, jint);
  void* (*GetDirectBufferAddress)(JNIEnv*, jobject);
  jlong (*GetDirectBufferCapacity)(JNIEnv*, jobject);
};
#endif

/*
 * jni.h — TEST DOUBLE of the JNI interface, for tests/jni/jni_harness.cpp only.
 *
 * This image has no JDK, so the JNI binding src/main/native/sux_jni.c could never be compiled
 * against the real header.  This file declares the part of the JNI C interface that sux_jni.c
 * uses — the types, constants and the JNINativeInterface_ / JNIInvokeInterface_ members it calls
 * — with the JNI specification's signatures and member names, so the unchanged sux_jni.c compiles
 * against it and the harness can drive every native method through an in-process fake JVM
 * (byte/int/long arrays, strings, direct ByteBuffers, exceptions, the Bootstrap callback).
 * The function tables here are NOT laid out like a real JVM's: a build for the JVM uses the
 * JDK's jni.h (src/main/native/Makefile, JAVA_HOME).  Nothing under sparkucx_amd/ includes it.
 */
#ifndef SUX_TEST_JNI_H
#define SUX_TEST_JNI_H

#include <stdarg.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef unsigned char jboolean;
typedef signed char jbyte;
typedef int jint;
typedef long jlong; /* LP64, as jni_md.h on Linux x86-64 */
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jobject jthrowable;
struct _jmethodID;
typedef struct _jmethodID* jmethodID;

#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_OK 0
#define JNI_ERR (-1)
#define JNI_EDETACHED (-2)
#define JNI_ABORT 2
#define JNI_VERSION_1_8 0x00010008

struct JNINativeInterface_;
struct JNIInvokeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
typedef const struct JNIInvokeInterface_* JavaVM;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv* env, const char* name);
  jint (*Throw)(JNIEnv* env, jthrowable obj);
  jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
  jboolean (*ExceptionCheck)(JNIEnv* env);
  void (*ExceptionClear)(JNIEnv* env);
  jobject (*NewGlobalRef)(JNIEnv* env, jobject lobj);
  void (*DeleteGlobalRef)(JNIEnv* env, jobject gref);
  jobject (*NewObject)(JNIEnv* env, jclass clazz, jmethodID methodID, ...);
  jclass (*GetObjectClass)(JNIEnv* env, jobject obj);
  jmethodID (*GetMethodID)(JNIEnv* env, jclass clazz, const char* name, const char* sig);
  jobject (*CallObjectMethod)(JNIEnv* env, jobject obj, jmethodID methodID, ...);
  jstring (*NewStringUTF)(JNIEnv* env, const char* utf);
  const char* (*GetStringUTFChars)(JNIEnv* env, jstring str, jboolean* isCopy);
  void (*ReleaseStringUTFChars)(JNIEnv* env, jstring str, const char* chars);
  jsize (*GetArrayLength)(JNIEnv* env, jarray array);
  jbyteArray (*NewByteArray)(JNIEnv* env, jsize len);
  jintArray (*NewIntArray)(JNIEnv* env, jsize len);
  jlongArray (*NewLongArray)(JNIEnv* env, jsize len);
  jbyte* (*GetByteArrayElements)(JNIEnv* env, jbyteArray array, jboolean* isCopy);
  jint* (*GetIntArrayElements)(JNIEnv* env, jintArray array, jboolean* isCopy);
  jlong* (*GetLongArrayElements)(JNIEnv* env, jlongArray array, jboolean* isCopy);
  void (*ReleaseByteArrayElements)(JNIEnv* env, jbyteArray array, jbyte* elems, jint mode);
  void (*ReleaseIntArrayElements)(JNIEnv* env, jintArray array, jint* elems, jint mode);
  void (*ReleaseLongArrayElements)(JNIEnv* env, jlongArray array, jlong* elems, jint mode);
  void (*GetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, jbyte* buf);
  void (*GetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, jint* buf);
  void (*SetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len,
                             const jbyte* buf);
  void (*SetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len,
                            const jint* buf);
  void (*SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len,
                             const jlong* buf);
  jint (*GetJavaVM)(JNIEnv* env, JavaVM** vm);
  void* (*GetDirectBufferAddress)(JNIEnv* env, jobject buf);
  jlong (*GetDirectBufferCapacity)(JNIEnv* env, jobject buf);
};

struct JNIInvokeInterface_ {
  jint (*AttachCurrentThread)(JavaVM* vm, void** penv, void* args);
  jint (*DetachCurrentThread)(JavaVM* vm);
  jint (*GetEnv)(JavaVM* vm, void** penv, jint version);
};

#ifdef __cplusplus
}
#endif
#endif

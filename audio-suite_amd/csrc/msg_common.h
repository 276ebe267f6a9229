// msg_common.h — shared macros for host/device code of libmsgpu.
#pragma once
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MSG_HD __host__ __device__ __forceinline__
#define MSG_DEV __device__ __forceinline__
#define MSG_NOINL __device__ __noinline__
#else
#define MSG_HD inline
#define MSG_DEV inline
#define MSG_NOINL
#endif

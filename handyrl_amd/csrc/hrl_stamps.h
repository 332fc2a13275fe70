// hrl_stamps.h — in-kernel clock stamps for diagnostic builds (tools/stamps.py).
#ifndef HRL_STAMPS_H
#define HRL_STAMPS_H

// Diagnostic build only (tools/stamps.py builds with -DHRL_STAMPS; libhrl.so never does): lane 0 of
// every workgroup writes the shader clock after draining its outstanding memory operations, so a
// wave's timeline splits into phases.  The drain serialises what the product overlaps.
#ifdef HRL_STAMPS
#define HRL_STAMP_DECL static __device__ unsigned long long *g_hrl_stamps = nullptr;
#define HRL_STAMP(k)                                                                                  \
    do {                                                                                              \
        __builtin_amdgcn_s_waitcnt(0);                                                                \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                   \
        if (threadIdx.x == 0 && g_hrl_stamps) g_hrl_stamps[(size_t)blockIdx.x * 16 + (k)] = t_;      \
    } while (0)
#define HRL_STAMP_WALL(k)                                                                             \
    do {                                                                                              \
        const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                               \
        if (threadIdx.x == 0 && g_hrl_stamps) g_hrl_stamps[(size_t)blockIdx.x * 16 + (k)] = t_;      \
    } while (0)
#else
#define HRL_STAMP_DECL
#define HRL_STAMP(k) do { } while (0)
#define HRL_STAMP_WALL(k) do { } while (0)
#endif

#endif  // HRL_STAMPS_H

// yk_api.h - host-side helpers shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>

#include "yacht_hip.h"

namespace yk {
void set_hip_error(hipError_t e);
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int grid_for(long n, int per_block) { return (int)((n + per_block - 1) / per_block); }
}  // namespace yk

#define YK_HIP(call)                                   \
    do {                                               \
        hipError_t e_ = (call);                        \
        if (e_ != hipSuccess) {                        \
            yk::set_hip_error(e_);                     \
            return YK_ERR_HIP;                         \
        }                                              \
    } while (0)

#define YK_LAUNCHED()                                  \
    do {                                               \
        hipError_t e_ = hipGetLastError();             \
        if (e_ != hipSuccess) {                        \
            yk::set_hip_error(e_);                     \
            return YK_ERR_HIP;                         \
        }                                              \
    } while (0)

// yk_api.h - host-side helpers shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>

#include "yacht_hip.h"

namespace yk {
void set_hip_error(hipError_t e);
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int grid_for(long n, int per_block) { return (int)((n + per_block - 1) / per_block); }

// The packed trajectory record image of one engine batch (yk_engine_pack_records), shared by
// the engine (writer) and the replay kernels (reader): 8 parts, each padded to 16 B -
// states[E][M] (64 B) | info[E][M][8] i32 | ctr[E][M][2] u64 | values[E][M] f64 |
// visits[E][VCAP] u32 | visits_off[E][M+1] i32 | n_moves[E] i32 | final[E] (64 B).
enum { REC_STATES, REC_INFO, REC_CTR, REC_VALUES, REC_VISITS, REC_VOFF, REC_NMOVES, REC_FINAL, REC_PARTS };
struct RecordLayout {
    int64_t off[REC_PARTS], bytes[REC_PARTS], total;
};
inline int64_t record_vcap(int64_t M, int64_t sims) { return 2 * M * (sims > 32 ? sims : 32); }
inline RecordLayout record_layout(int64_t E, int64_t M, int64_t VCAP) {
    RecordLayout L;
    const int64_t b[REC_PARTS] = {E * M * 64, E * M * 8 * 4, E * M * 2 * 8, E * M * 8,
                                  E * VCAP * 4, E * (M + 1) * 4, E * 4, E * 64};
    int64_t off = 0;
    for (int i = 0; i < REC_PARTS; i++) {
        L.off[i] = off;
        L.bytes[i] = b[i];
        off += (b[i] + 15) & ~15LL;
    }
    L.total = off;
    return L;
}
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

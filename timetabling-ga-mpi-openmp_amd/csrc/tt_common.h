// Shared device-side definitions for the ttga HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ttga {

constexpr int kSlots = 45;             // Solution.cpp:52,57
constexpr int kSlotsPerDay = 9;
constexpr int kMaxRooms = 64;          // rooms are bitmasks in one 64-bit word
constexpr int kMaxSlotEvents = 256;    // per-slot event bitsets (4 x 64 bits) in the matcher

// slot s is the last of its day (s % 9 == 8): Solution.cpp:94
constexpr uint64_t kLastSlotMask = (1ull << 8) | (1ull << 17) | (1ull << 26) | (1ull << 35) | (1ull << 44);
// bit k set iff slots k, k+1, k+2 lie in one day (k % 9 <= 6): the >2-in-a-row window
constexpr uint64_t kTripleMask = 0x7Full | (0x7Full << 9) | (0x7Full << 18) | (0x7Full << 27) | (0x7Full << 36);

// Device image of a Problem (Problem.h:35-46), read-only for the handle's lifetime.
struct DevProblem {
    int E, R, S, EW;              // EW = 32-bit words per correlation row
    const int32_t* sn;            // [E] studentNumber
    const int32_t* stu_off;       // [S+1] CSR of student_events by student
    const int32_t* stu_ev;        //   events of each student, ascending
    const int32_t* ev_off;        // [E+1] CSR by event
    const int32_t* ev_stu;        //   students of each event, ascending
    const uint64_t* poss;         // [E] possibleRooms as room bitmasks
    const uint32_t* corr;         // [E*EW] eventCorrelations bit-matrix (diagonal included)
    int EW64;                     // 64-bit words per event bitset
    const uint64_t* cupT;         // [EW64][E] upper-triangle correlation bits, word-major:
                                  //   cupT[w*E+i] bit b <=> corr(i, 64w+b) and 64w+b > i
    const uint64_t* corr64;       // [E][EW64] full eventCorrelations rows (diagonal included)
    const int32_t* stc_off;       // [S+1] per-student event lists padded to multiples of 8
    const int32_t* stc_ev;        //   padding entries hold E (a sentinel column)
    const uint32_t* sid;          // lane-phase student lists, students sorted by padded size:
                                  //   each student's events as u16 ids, padded to an even count
                                  //   with E (the sentinel column); 64 B of slack at the end
    const int4* srun;             // runs of equal-size students: (ids per student, first dword
                                  //   in sid, students, 0); a wave's runs are contiguous
    const int32_t* srun_part;     // run index range of each wave: [kSrunPart4 + w] for 4-wave,
                                  //   [kSrunPart8 + w] for 8-wave, [kSrunPart16 + w] for 16-wave groups
    int32_t* status;              // device status word (tt_device_status)
};
constexpr int kSrunPart4 = 0, kSrunPart8 = 5, kSrunPart16 = 14, kSrunPartLen = 32;
__host__ __device__ constexpr int srun_part_base(int nw) { return nw == 4 ? kSrunPart4 : nw == 8 ? kSrunPart8 : kSrunPart16; }

// Park-Miller "minimal standard" generator, Schrage's method
// (Random.h:15-19, Random.cc:27-37). Bit-exact with the reference: int64
// state arithmetic, then AM * state in IEEE fp64 (gfx950 has full fp64).
// Every state after the first draw lies in [0, 2^31 - 1), where Schrage's
// steps fit 32-bit integers exactly (16807 * 127772 < 2^31 - 1), so the
// 64-bit form is only needed for an out-of-range initial seed.
__device__ __forceinline__ double pm_next(int64_t& s) {
    const int64_t IA = 16807, IM = 2147483647, IQ = 127773, IR = 2836;
    const double AM = 1.0 / 2147483647.0;
    if ((uint64_t)s <= 0x7FFFFFFFull) {
        const uint32_t u = (uint32_t)s;
        const uint32_t k32 = u / 127773u;
        int32_t t = 16807 * (int32_t)(u - k32 * 127773u) - 2836 * (int32_t)k32;
        if (t < 0) t += 2147483647;
        s = t;
        return __dmul_rn(AM, (double)t);
    }
    int64_t k = s / IQ;
    s = IA * (s - k * IQ) - IR * k;
    if (s < 0) s += IM;
    return __dmul_rn(AM, (double)s);
}

// Park-Miller jump: a * b mod (2^31 - 1) for a, b < 2^31 - 1. For an in-range
// state s (every state after the first draw), k Schrage steps give exactly
// s * 16807^k mod (2^31 - 1).
constexpr uint32_t kPmM = 2147483647u;
__device__ __forceinline__ uint32_t pm_mulmod(uint32_t a, uint32_t b) {
    const uint64_t p = (uint64_t)a * b;
    const uint32_t r = (uint32_t)(p & kPmM) + (uint32_t)(p >> 31);
    return r >= kPmM ? r - kPmM : r;
}
// 16807^(n) mod (2^31 - 1)
__device__ __forceinline__ uint32_t pm_pow(int n) {
    uint32_t r = 1, b = 16807u;
    for (; n; n >>= 1) {
        if (n & 1) r = pm_mulmod(r, b);
        b = pm_mulmod(b, b);
    }
    return r;
}

// (int)(next() * n): truncation of the fp64 product (Solution.cpp:52, ga.cpp:135)
__device__ __forceinline__ int pm_pick(int64_t& s, int n) { return (int)__dmul_rn(pm_next(s), (double)n); }

// >2 in a row + single class of one student's attendance mask m, the 45-bit set
// of slots the student attends (Solution.cpp:99-137)
__device__ __forceinline__ int mask_scv(uint64_t m) {
    int sc = __popcll(m & (m >> 1) & (m >> 2) & kTripleMask);
#pragma unroll
    for (int d = 0; d < 5; ++d) sc += (__popc((uint32_t)(m >> (9 * d)) & 0x1FFu) == 1);
    return sc;
}

// Full-wave sum (every lane active): DPP row shifts + readlane, no LDS round
// trips. Written out rather than __reduce_add_sync, whose library reduction
// also carries a partial-EXEC path at every call site (code size: the local
// search inlines it dozens of times).
#ifndef TT_WAVE_SUM_BCAST
#define TT_WAVE_SUM_BCAST 1
#endif
__device__ __forceinline__ int wave_sum(int v) {
#if TT_WAVE_SUM_BCAST
    // row_shr 1/2/4/8 leave row r's sum in lane 16r + 15; row_bcast:15 adds row r's
    // into row r+1 (rows 1, 3), row_bcast:31 lane 31's into rows 2-3: lane 63 holds
    // the wave's sum -- one readlane instead of four plus three scalar adds
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);    // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);    // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);    // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);    // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15 (rows 1, 3)
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31 (rows 2, 3)
    return __builtin_amdgcn_readlane(v, 63);
#else
    v += __builtin_amdgcn_update_dpp(0, v, 0x101, 0xf, 0xf, true);    // row_shl:1 (lane i += lane i+1)
    v += __builtin_amdgcn_update_dpp(0, v, 0x102, 0xf, 0xf, true);    // row_shl:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x104, 0xf, 0xf, true);    // row_shl:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x108, 0xf, 0xf, true);    // row_shl:8: lane 16r holds row r's sum
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
#endif
}

// Wave ballot / any of a bool: the builtin takes the compare's lane mask as
// it is (HIP's __ballot(int) first turns the bool into 0/1 in a VGPR and
// compares it again: two more VALU per ballot).
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0ull; }

// Index of this thread's wave in the workgroup, as a wave-uniform (SGPR) value
// so that loops and loads driven by it stay scalar.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

}  // namespace ttga

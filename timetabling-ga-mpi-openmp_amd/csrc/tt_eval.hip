// Batched fitness evaluation: Solution::computeFeasibility / computeHcv /
// computeScv / computePenalty (Solution.cpp:63-170) for a device-resident
// population slot[P][E], room[P][E].
//
// Closed forms (proven equal to the reference's loops
// on the golden vectors):
//   scv = sum_e [slot_e % 9 == 8] * studentNumber[e]                    (last slot)
//       + sum_s popcount(m_s & m_s>>1 & m_s>>2 & triple-window)         (>2 in a row)
//       + sum_s sum_d [popcount(m_s day d) == 1]                        (single class)
//     where m_s is the 45-bit set of slots student s attends;
//   hcv = sum_cells C(n_cell, 2)           (same slot and room)
//       + #{i<j : slot_i == slot_j, corr_ij}
//       + #{e : room_e not possible for e};
//   feasible <=> hcv == 0 (Solution.cpp:63-84 tests the same three conditions).
//
// Two kernels:
//  * eval_tile (E <= 1024): one workgroup per tile of 64 individuals, mixing a
//    lane-per-individual phase (attendance masks) with a wave-per-individual
//    phase (bitset hcv terms); see below.
//  * eval_block (any E): one 256-thread workgroup per individual; slot
//    buckets in LDS enumerate only same-slot pairs for the correlation term.
#include <algorithm>
#include <type_traits>

#include "tt_internal.h"

namespace ttga {

// ---------------------------------------------------------------- eval_tile
// One workgroup of kTileWaves waves per tile of 64 individuals (persistent
// over tiles). The tile's slot rows sit in LDS with an odd-dword row stride
// plus a sentinel column E (slot 63, outside every day mask).
//  * lane phase (LANE = INDIVIDUAL): wave w builds the 45-bit attendance mask
//    of students w, w+8, ... from 8-padded event lists (8 independent
//    conflict-free ds_read_u8 per chunk) -> >2-in-a-row and single-class terms;
//  * wave phase (WAVE = INDIVIDUAL): per-slot event bitsets B[t] (ds_or_b64),
//    room-cell counters (ds_add_rtn), unsuitable rooms, last-slot term, and the
//    correlated same-slot pairs as popcount(cupT[w][i] & B[slot_i][w]) over the
//    upper-triangle words (1.6 K word ops per individual at E=400 instead of
//    13 K neighbour lookups).


struct TileLayout {
    int SP;           // tile row stride (bytes)
    int WS;           // per-wave scratch bytes
    size_t off_wave;  // start of per-wave scratch
    size_t off_part;  // [kTileWaves][64] lane-phase partials, then hq[64], sq[64]
    size_t bytes;
};

__host__ __device__ inline TileLayout tile_layout(int E, int R) {
    TileLayout L;
    int sp = (E + 1 + 3) & ~3;                 // room for the sentinel column
    if (((sp >> 2) & 1) == 0) sp += 4;         // odd dword stride: conflict-free column reads
    L.SP = sp;
    const int ew64 = (E + 63) / 64;
    L.WS = (kSlots * ew64 * 8 + kSlots * R * 4 + 15) & ~15;
    L.off_wave = ((size_t)64 * sp + 15) & ~(size_t)15;
    L.off_part = L.off_wave + (size_t)kTileWaves * L.WS;
    L.bytes = L.off_part + 4 * (size_t)(kTileWaves * 64 + 128);
    return L;
}

// EWC > 0: compile-time number of 64-event words (E <= 64*EWC); the per-event
// invariants of a lane's events (possible rooms, studentNumber, the upper-
// triangle correlation words) live in registers for the whole launch, so an
// individual costs only its own slot/room reads plus LDS traffic.
// EWC == 0: runtime word count, invariants re-read from global memory.
template <int EWC>
__global__ __launch_bounds__(64 * kTileWaves) void eval_tile_kernel(DevProblem pb, const uint8_t* __restrict__ slot,
                                                                     const uint8_t* __restrict__ room, int P,
                                                                     int32_t* __restrict__ hcv_out,
                                                                     int32_t* __restrict__ scv_out,
                                                                     uint8_t* __restrict__ feas_out,
                                                                     int32_t* __restrict__ pen_out, int ablate) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int E = pb.E, R = pb.R;
    const int EW64 = EWC > 0 ? EWC : pb.EW64;
    const int lane = threadIdx.x & 63, wv = wave_id();
    const TileLayout L = tile_layout(E, R);
    // ablate (profiling only, results invalid): 1 skip lane phase, 2 skip wave phase, 4 skip corr words
    const int SP = L.SP;
    uint8_t* tile = lds;
    uint64_t* B = (uint64_t*)(lds + L.off_wave + (size_t)wv * L.WS);   // [45][EW64]
    uint32_t* cnt = (uint32_t*)(B + kSlots * EW64);                     // [45*R]
    int32_t* part = (int32_t*)(lds + L.off_part);                       // [kTileWaves][64]
    int32_t* hq = part + kTileWaves * 64;                               // [64]
    int32_t* sq = hq + 64;                                              // [64]
    const int tiles = (P + 63) / 64;
    const int nthr = 64 * kTileWaves;

    constexpr int NR = EWC > 0 ? EWC : 1;
    uint64_t inv_poss[NR], inv_cup[NR][NR];
    int inv_sn[NR];
    if constexpr (EWC > 0) {
#pragma unroll
        for (int r = 0; r < EWC; ++r) {
            const int e = lane + 64 * r;
            const bool ok = e < E;
            inv_poss[r] = ok ? pb.poss[e] : ~0ull;
            inv_sn[r] = ok ? pb.sn[e] : 0;
#pragma unroll
            for (int w = 0; w < EWC; ++w) inv_cup[r][w] = (w >= r && ok) ? pb.cupT[(size_t)w * E + e] : 0ull;
        }
    }

    for (int tl = blockIdx.x; tl < tiles; tl += gridDim.x) {
        const long p0 = (long)tl * 64;
        const int np = (int)min((long)64, (long)P - p0);
        __syncthreads();
        // ---- stage slot rows + sentinel column
        const uint8_t* src = slot + p0 * E;
        if ((E & 3) == 0) {
            const int wpr = E >> 2;
            const uint32_t* s32 = (const uint32_t*)src;
            for (int w = threadIdx.x; w < np * wpr; w += nthr) {
                const int r = w / wpr, c = w - r * wpr;
                *(uint32_t*)(tile + r * SP + 4 * c) = s32[w];
            }
        } else {
            for (int b = threadIdx.x; b < np * E; b += nthr) {
                const int r = b / E, c = b - r * E;
                tile[r * SP + c] = src[b];
            }
        }
        if (threadIdx.x < 64) tile[threadIdx.x * SP + E] = 63;
        __syncthreads();

        // ---- lane phase: per-student attendance masks (Solution.cpp:98-137)
        if (!(ablate & 1)) {
            // this wave's students as one stream of 8-id chunk records; the next
            // record is loaded while the current one's 8 LDS reads are in flight
            const uint8_t* my = tile + lane * SP;
            int sc = 0;
            const int c0 = pb.wch_off[wv], c1 = pb.wch_off[wv + 1];
            if (c0 < c1) {
                uint4 cur = pb.wch[c0];
                uint64_t m = 0;
                for (int c = c0; c < c1; ++c) {
                    const uint4 nxt = pb.wch[c + 1 < c1 ? c + 1 : c];
                    const uint32_t w[4] = {cur.x, cur.y, cur.z, cur.w};
                    uint32_t sl[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) sl[j] = my[(w[j >> 1] >> (16 * (j & 1))) & 0x7FFFu];
#pragma unroll
                    for (int j = 0; j < 8; ++j) m |= 1ull << (sl[j] & 63);
                    if (cur.x & 0x8000u) {                       // last chunk of a student
                        sc += __popcll(m & (m >> 1) & (m >> 2) & kTripleMask);
#pragma unroll
                        for (int d = 0; d < 5; ++d) sc += (__popc((uint32_t)(m >> (9 * d)) & 0x1FFu) == 1);
                        m = 0;
                    }
                    cur = nxt;
                }
            }
            part[wv * 64 + lane] = sc;
        }

        // ---- wave phase: hcv terms + last-slot term, one individual per wave at a time
        for (int q = wv; q < ((ablate & 2) ? 0 : np); q += kTileWaves) {
            for (int c = lane; c < kSlots * EW64; c += 64) B[c] = 0ull;
            for (int c = lane; c < kSlots * R; c += 64) cnt[c] = 0u;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint8_t* rs = tile + q * SP;
            const uint8_t* rr = room + (p0 + q) * E;
            int h = 0, last = 0;
            bool bad = false;
            if constexpr (EWC > 0) {
                uint32_t sv[EWC], rv[EWC];
#pragma unroll
                for (int r = 0; r < EWC; ++r) {
                    const int e = lane + 64 * r;
                    sv[r] = e < E ? rs[e] : 0u;
                    rv[r] = e < E ? rr[e] : 0u;
                }
#pragma unroll
                for (int r = 0; r < EWC; ++r) {
                    if (lane + 64 * r < E) {
                        const int s = sv[r], ro = rv[r];
                        if (s >= kSlots || ro >= R) {
                            bad = true;
                        } else {
                            atomicOr((unsigned long long*)&B[s * EWC + r], 1ull << lane);
                            h += (int)atomicAdd(&cnt[s * R + ro], 1u);                 // Solution.cpp:148-150
                            h += (int)(((inv_poss[r] >> ro) & 1ull) ^ 1ull);            // :155-156
                            last += inv_sn[r] * (int)((kLastSlotMask >> s) & 1ull);     // :93-96
                        }
                    }
                }
                const bool any_bad = __any(bad);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (!any_bad && !(ablate & 4)) {
#pragma unroll
                    for (int r = 0; r < EWC; ++r) {                                     // :151-153
                        if (lane + 64 * r < E) {
                            const uint64_t* brow = B + sv[r] * EWC;
#pragma unroll
                            for (int w = r; w < EWC; ++w) h += __popcll(inv_cup[r][w] & brow[w]);
                        }
                    }
                }
                bad = any_bad;
            } else {
                for (int e = lane; e < E; e += 64) {
                    const int s = rs[e], r = rr[e];
                    if (s >= kSlots || r >= R) { bad = true; continue; }
                    atomicOr((unsigned long long*)&B[s * EW64 + (e >> 6)], 1ull << (e & 63));
                    h += (int)atomicAdd(&cnt[s * R + r], 1u);
                    h += (int)(((pb.poss[e] >> r) & 1ull) ^ 1ull);
                    last += pb.sn[e] * (int)((kLastSlotMask >> s) & 1ull);
                }
                const bool any_bad = __any(bad);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (!any_bad && !(ablate & 4)) {
                    for (int i = lane; i < E; i += 64) {
                        const uint64_t* brow = B + rs[i] * EW64;
                        for (int w = i >> 6; w < EW64; ++w) h += __popcll(pb.cupT[(size_t)w * E + i] & brow[w]);
                    }
                }
                bad = any_bad;
            }
            h = wave_sum(h);
            last = wave_sum(last);
            if (lane == 0) { hq[q] = bad ? -1 : h; sq[q] = last; }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        __syncthreads();
        if (wv == 0 && lane < np) {
            const long p = p0 + lane;
            const int h = hq[lane];
            if (h < 0) {
                hcv_out[p] = -1; scv_out[p] = -1; feas_out[p] = 0; pen_out[p] = -1;
            } else {
                int sc = sq[lane];
#pragma unroll
                for (int w = 0; w < kTileWaves; ++w) sc += part[w * 64 + lane];
                hcv_out[p] = h;
                scv_out[p] = sc;
                feas_out[p] = h == 0 ? 1 : 0;
                pen_out[p] = h == 0 ? sc : 1000000 + h;
            }
        }
    }
}

// ---------------------------------------------------------------- eval_tile4
// Second-generation tile kernel: NW waves per 64-individual tile, sized so that
// at E = 400 four workgroups (16 waves) fit one CU and a 65,536-member
// population is one tile per workgroup.
//  * lane-phase records come through the scalar cache (s_load_dwordx4 via the
//    constant address space) from a student-ordered stream; wave w owns a
//    contiguous student range balanced by record count;
//  * the wave phase prefetches the next individual's room row while the
//    current one is scored; cell counters are packed u16 pairs;
//  * PK selects how a lane keeps possibleRooms/studentNumber of its events:
//    1 = one packed register (R <= 16, studentNumber < 65536), 2 = u32 mask
//    (R <= 32), 0 = u64 mask.
typedef __attribute__((address_space(4))) const uint32_t ConstU32;
typedef __attribute__((address_space(4))) const int32_t ConstI32;

struct Tile4Layout {
    int SP, WS;
    size_t off_wave, off_part, bytes;
};

__host__ __device__ inline Tile4Layout tile4_layout(int E, int R, int NW) {
    Tile4Layout L;
    int sp = (E + 1 + 3) & ~3;
    if (((sp >> 2) & 1) == 0) sp += 4;
    L.SP = sp;
    const int ew64 = (E + 63) / 64;
    const int cntw = (kSlots * R + 1) / 2;
    L.WS = (kSlots * ew64 * 8 + cntw * 4 + 15) & ~15;
    L.off_wave = ((size_t)64 * sp + 15) & ~(size_t)15;
    L.off_part = L.off_wave + (size_t)NW * L.WS;
    L.bytes = L.off_part + 4 * (size_t)(NW * 64 + 64);
    return L;
}

template <int EWC, int NW, int PK>
__global__ __launch_bounds__(64 * NW, 16 / NW) void eval_tile4_kernel(DevProblem pb, const uint8_t* __restrict__ slot,
                                                              const uint8_t* __restrict__ room, int P,
                                                              int32_t* __restrict__ hcv_out,
                                                              int32_t* __restrict__ scv_out,
                                                              uint8_t* __restrict__ feas_out,
                                                              int32_t* __restrict__ pen_out, int ablate) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int NT = 64 * NW;
    const int E = pb.E, R = pb.R;
    const int lane = threadIdx.x & 63, wv = wave_id();
    const Tile4Layout L = tile4_layout(E, R, NW);
    const int SP = L.SP;
    uint8_t* tile = lds;
    uint8_t* ws = lds + L.off_wave + (size_t)wv * L.WS;
    uint64_t* B = (uint64_t*)ws;                              // [45][EWC] event bitsets per slot
    uint32_t* cnt = (uint32_t*)(B + kSlots * EWC);            // [45*R] u16 cell counters, 2 per dword
    int32_t* part = (int32_t*)(lds + L.off_part);             // [NW][64] scv partials
    int32_t* hq = part + NW * 64;                             // [64] hcv (or -1)
    const int tiles = (P + 63) / 64;

    // per-event invariants of this lane's events e = lane + 64 r
    using PossT = typename std::conditional<PK == 0, uint64_t, uint32_t>::type;
    uint64_t inv_cup[EWC][EWC];
    PossT inv_poss[EWC];
    uint32_t inv_ps[EWC];
    int inv_sn[EWC];
#pragma unroll
    for (int r = 0; r < EWC; ++r) {
        const int e = lane + 64 * r;
        const bool ok = e < E;
        if constexpr (PK == 1) {
            inv_ps[r] = ok ? ((uint32_t)pb.poss[e] | ((uint32_t)pb.sn[e] << 16)) : 0xFFFFu;
        } else {
            inv_poss[r] = ok ? (PossT)pb.poss[e] : (PossT)~0ull;
            inv_sn[r] = ok ? pb.sn[e] : 0;
        }
#pragma unroll
        for (int w = 0; w < EWC; ++w) inv_cup[r][w] = (w >= r && ok) ? pb.cupT[(size_t)w * E + e] : 0ull;
    }
    const ConstU32* rec = (const ConstU32*)pb.sch;
    const ConstI32* ptab = (const ConstI32*)pb.sch_part;
    const int pbase = NW == 4 ? kSchPart4 : kSchPart8;
    const int c0 = ptab[pbase + wv], c1 = ptab[pbase + wv + 1];
    const bool wide = (E & 15) == 0 && (((uintptr_t)slot) & 15) == 0;
    const int qpr = E >> 4;
    const uint32_t qinv = ((1u << 20) + (uint32_t)qpr - 1) / (uint32_t)max(qpr, 1);   // w / qpr for w < 2^12

    for (int tl = blockIdx.x; tl < tiles; tl += gridDim.x) {
        const long p0 = (long)tl * 64;
        const int np = (int)min((long)64, (long)P - p0);
        __syncthreads();
        // ---- stage the tile's slot rows (+ sentinel column E = slot 63)
        const uint8_t* src = slot + p0 * E;
        if (wide) {
            const uint4* s16 = (const uint4*)src;
#pragma unroll 2
            for (int w = threadIdx.x; w < np * qpr; w += NT) {
                const int r = (int)(((uint32_t)w * qinv) >> 20), c = w - r * qpr;
                const uint4 v = s16[w];
                uint32_t* d = (uint32_t*)(tile + r * SP + 16 * c);
                d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
            }
        } else {
#pragma unroll 1
            for (int r = wv; r < np; r += NW)
#pragma unroll 1
                for (int c = lane; c < E; c += 64) tile[r * SP + c] = src[(long)r * E + c];
        }
        if (threadIdx.x < 64) tile[threadIdx.x * SP + E] = 63;
        __syncthreads();

        // ---- lane phase (lane = individual): attendance masks of this wave's students
        int sc = 0;
        if (!(ablate & 1) && c0 < c1) {
            const uint8_t* my = tile + lane * SP;
            uint32_t cur[4] = {rec[4 * c0], rec[4 * c0 + 1], rec[4 * c0 + 2], rec[4 * c0 + 3]};
            uint64_t m = 0;
            for (int c = c0; c < c1; ++c) {
                const int cn = c + 1 < c1 ? c + 1 : c;
                const uint32_t nxt[4] = {rec[4 * cn], rec[4 * cn + 1], rec[4 * cn + 2], rec[4 * cn + 3]};
                const uint32_t* w = cur;
                uint32_t sl[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) sl[j] = my[(w[j >> 1] >> (16 * (j & 1))) & 0x7FFFu];
#pragma unroll
                for (int j = 0; j < 8; ++j) m |= 1ull << (sl[j] & 63);
                if (cur[0] & 0x8000u) {                                  // last record of a student
                    sc += __popcll(m & (m >> 1) & (m >> 2) & kTripleMask);   // Solution.cpp:99-117
#pragma unroll
                    for (int d = 0; d < 5; ++d) sc += (__popc((uint32_t)(m >> (9 * d)) & 0x1FFu) == 1);   // :119-137
                    m = 0;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
            }
        }
        part[wv * 64 + lane] = sc;

        // ---- wave phase (wave = individual): hcv terms + last-slot term
        const int nq = (ablate & 2) ? 0 : np;
        uint32_t rvn[EWC];
#pragma unroll
        for (int r = 0; r < EWC; ++r) rvn[r] = 0u;
        if (wv < nq) {
            const uint8_t* rr = room + (p0 + wv) * E;
#pragma unroll
            for (int r = 0; r < EWC; ++r) rvn[r] = lane + 64 * r < E ? rr[lane + 64 * r] : 0u;
        }
        for (int q = wv; q < nq; q += NW) {
            uint32_t rv[EWC], sv[EWC];
#pragma unroll
            for (int r = 0; r < EWC; ++r) rv[r] = rvn[r];
            if (q + NW < nq) {                                          // prefetch the next room row
                const uint8_t* rr = room + (p0 + q + NW) * E;
#pragma unroll
                for (int r = 0; r < EWC; ++r) rvn[r] = lane + 64 * r < E ? rr[lane + 64 * r] : 0u;
            }
            for (int c = lane; c < (L.WS >> 4); c += 64) ((uint4*)ws)[c] = make_uint4(0u, 0u, 0u, 0u);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint8_t* rs = tile + q * SP;
#pragma unroll
            for (int r = 0; r < EWC; ++r) sv[r] = lane + 64 * r < E ? rs[lane + 64 * r] : 0u;
            int h = 0, last = 0;
            bool bad = false;
#pragma unroll
            for (int r = 0; r < EWC; ++r) {
                if (lane + 64 * r < E) {
                    const uint32_t s = sv[r], ro = rv[r];
                    if (s >= (uint32_t)kSlots || ro >= (uint32_t)R) {
                        bad = true;
                    } else {
                        atomicOr((unsigned long long*)&B[s * EWC + r], 1ull << lane);
                        const uint32_t cell = s * R + ro, sh = (cell & 1u) << 4;
                        const uint32_t old = atomicAdd(&cnt[cell >> 1], 1u << sh);
                        h += (int)((old >> sh) & 0xFFFFu);                               // Solution.cpp:148-150
                        const bool last_slot = (kLastSlotMask >> s) & 1ull;
                        if constexpr (PK == 1) {
                            h += (int)(((inv_ps[r] >> ro) & 1u) ^ 1u);                  // :155-156
                            last += last_slot ? (int)(inv_ps[r] >> 16) : 0;             // :93-96
                        } else {
                            h += (int)(((inv_poss[r] >> ro) & 1u) ^ 1u);
                            last += last_slot ? inv_sn[r] : 0;
                        }
                    }
                }
            }
            const bool any_bad = __any(bad);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (!any_bad && !(ablate & 4)) {
#pragma unroll
                for (int r = 0; r < EWC; ++r) {                                         // :151-153
                    if (lane + 64 * r < E) {
                        const uint64_t* brow = B + sv[r] * EWC;
#pragma unroll
                        for (int w = r; w < EWC; ++w) h += __popcll(inv_cup[r][w] & brow[w]);
                    }
                    if (r & 1) __builtin_amdgcn_sched_barrier(0);   // bound the B words in flight (VGPRs)
                }
            }
            h = wave_sum(h);
            last = wave_sum(last);
            if (lane == 0) {
                hq[q] = any_bad ? -1 : h;
                part[wv * 64 + q] += last;
            }
        }
        __syncthreads();
        if (wv == 0 && lane < np) {
            const long p = p0 + lane;
            const int h = hq[lane];
            if (h < 0) {
                hcv_out[p] = -1; scv_out[p] = -1; feas_out[p] = 0; pen_out[p] = -1;
            } else {
                int s2 = 0;
#pragma unroll
                for (int w = 0; w < NW; ++w) s2 += part[w * 64 + lane];
                hcv_out[p] = h;
                scv_out[p] = s2;
                feas_out[p] = h == 0 ? 1 : 0;
                pen_out[p] = h == 0 ? s2 : 1000000 + h;
            }
        }
    }
}

// ---------------------------------------------------------------- eval_tile5
// Third-generation tile kernel. Same two phases as eval_tile4, rearranged so
// that the LDS holds either the tile or the wave workspaces, never both:
//  * lane phase as eval_tile4 (8-padded per-student records through the scalar
//    cache; a back-to-back record stream with per-entry end flags measured
//    slower: its uniform per-entry branches serialise the mask updates);
//  * after a workgroup barrier the tile is dead and its bytes become the
//    per-wave workspaces; the wave phase reads each individual's slot and
//    room rows straight from global memory (L2-hot: the staging loads just
//    touched them), one individual ahead;
//  * an individual with an invalid gene is detected from registers before any
//    LDS work (its outputs are the -1 sentinels anyway); the valid path has
//    no per-event branches except on the last, partial event word;
//  * CNT32: u32 cell counters (address = one mad); otherwise packed u16 pairs;
//  * B rows are read with single ds_read_b64 (lds_row_b64 below).

// LDS byte address of a pointer into dynamic shared memory.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// N consecutive 64-bit LDS words at byte address addr, as N single
// ds_read_b64 (the compiler would pair them into ds_read2_b64) with the wait
// in the same asm block, so the results are defined when it ends.
#define TT_RD(k, o) "ds_read_b64 %" #k ", %" #o " offset:" #k "*8\n"
template <int N>
__device__ __forceinline__ void lds_row_b64(uint32_t addr, uint64_t* v) {
    static_assert(N >= 1 && N <= 7, "1..7 words");
    uint64_t d[7];
    if constexpr (N == 7)
        asm volatile(TT_RD(0, 7) TT_RD(1, 7) TT_RD(2, 7) TT_RD(3, 7) TT_RD(4, 7) TT_RD(5, 7) TT_RD(6, 7) "s_waitcnt lgkmcnt(0)"
                     : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]), "=&v"(d[4]), "=&v"(d[5]), "=&v"(d[6])
                     : "v"(addr) : "memory");
    else if constexpr (N == 6)
        asm volatile(TT_RD(0, 6) TT_RD(1, 6) TT_RD(2, 6) TT_RD(3, 6) TT_RD(4, 6) TT_RD(5, 6) "s_waitcnt lgkmcnt(0)"
                     : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]), "=&v"(d[4]), "=&v"(d[5]) : "v"(addr) : "memory");
    else if constexpr (N == 5)
        asm volatile(TT_RD(0, 5) TT_RD(1, 5) TT_RD(2, 5) TT_RD(3, 5) TT_RD(4, 5) "s_waitcnt lgkmcnt(0)"
                     : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]), "=&v"(d[4]) : "v"(addr) : "memory");
    else if constexpr (N == 4)
        asm volatile(TT_RD(0, 4) TT_RD(1, 4) TT_RD(2, 4) TT_RD(3, 4) "s_waitcnt lgkmcnt(0)"
                     : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]), "=&v"(d[3]) : "v"(addr) : "memory");
    else if constexpr (N == 3)
        asm volatile(TT_RD(0, 3) TT_RD(1, 3) TT_RD(2, 3) "s_waitcnt lgkmcnt(0)"
                     : "=&v"(d[0]), "=&v"(d[1]), "=&v"(d[2]) : "v"(addr) : "memory");
    else if constexpr (N == 2)
        asm volatile(TT_RD(0, 2) TT_RD(1, 2) "s_waitcnt lgkmcnt(0)" : "=&v"(d[0]), "=&v"(d[1]) : "v"(addr) : "memory");
    else
        asm volatile(TT_RD(0, 1) "s_waitcnt lgkmcnt(0)" : "=&v"(d[0]) : "v"(addr) : "memory");
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = d[k];
}
#undef TT_RD

// Correlated same-slot pairs of the lane's events (word R onwards):
// h += popcount(cupT upper words & B[slot] words), one asm row read per event word.
template <int R, int EWC>
__device__ __forceinline__ void corr_words(uint32_t bbase, const uint32_t* sv, const uint64_t (*cup)[EWC], int lane,
                                           int E, bool last_partial, int& h) {
    if constexpr (R < EWC) {
        if (R < EWC - 1 || !last_partial || lane + 64 * R < E) {
            uint64_t bw[EWC - R];
            lds_row_b64<EWC - R>(bbase + sv[R] * (uint32_t)(EWC * 8) + 8 * R, bw);
#pragma unroll
            for (int w = R; w < EWC; ++w) h += __popcll(cup[R][w] & bw[w - R]);
        }
        corr_words<R + 1, EWC>(bbase, sv, cup, lane, E, last_partial, h);
    }
}

struct Tile5Layout {
    int SP, WS;
    size_t off_ws, off_part, bytes;
};

__host__ __device__ inline Tile5Layout tile5_layout(int E, int R, int NW, bool cnt32, bool alias) {
    Tile5Layout L;
    int sp = (E + 1 + 3) & ~3;
    if (((sp >> 2) & 1) == 0) sp += 4;
    L.SP = sp;
    const int ew64 = (E + 63) / 64;
    const int cntb = cnt32 ? kSlots * R * 4 : ((kSlots * R + 1) / 2) * 4;
    L.WS = (kSlots * ew64 * 8 + cntb + 15) & ~15;
    L.off_ws = alias ? 0 : (((size_t)64 * sp + 15) & ~(size_t)15);
    const size_t uni = alias ? std::max((size_t)64 * sp, (size_t)NW * L.WS) : L.off_ws + (size_t)NW * L.WS;
    L.off_part = (uni + 15) & ~(size_t)15;
    L.bytes = L.off_part + 4 * (size_t)(NW * 64 + 64);
    return L;
}

template <int EWC, int NW, bool CNT32, int PK, bool ALIAS>
__global__ __launch_bounds__(64 * NW, 4) void eval_tile5_kernel(DevProblem pb, const uint8_t* __restrict__ slot,
                                                              const uint8_t* __restrict__ room, int P,
                                                              int32_t* __restrict__ hcv_out,
                                                              int32_t* __restrict__ scv_out,
                                                              uint8_t* __restrict__ feas_out,
                                                              int32_t* __restrict__ pen_out, int ablate) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int NT = 64 * NW;
    const int E = pb.E, R = pb.R;
    const int lane = threadIdx.x & 63, wv = wave_id();
    const Tile5Layout L = tile5_layout(E, R, NW, CNT32, ALIAS);
    const int SP = L.SP;
    uint8_t* tile = lds;
    uint8_t* ws = lds + L.off_ws + (size_t)wv * L.WS;         // ALIAS: on top of the dead tile
    uint64_t* B = (uint64_t*)ws;                              // [45][EWC] event bitsets per slot
    uint32_t* cnt = (uint32_t*)(B + kSlots * EWC);            // cell counters
    int32_t* part = (int32_t*)(lds + L.off_part);             // [NW][64] scv partials
    int32_t* hq = part + NW * 64;                             // [64] hcv (or -1)
    const int tiles = (P + 63) / 64;
    const bool last_partial = E < 64 * EWC;                   // lanes of word EWC-1 beyond E

    // PK as in eval_tile4: 1 = possibleRooms | studentNumber << 16 in one register
    // (R <= 16, studentNumber < 65536), 2 = u32 mask (R <= 32), 0 = u64 mask
    using PossT = typename std::conditional<PK == 0, uint64_t, uint32_t>::type;
    uint64_t inv_cup[EWC][EWC];
    PossT inv_poss[EWC];
    uint32_t inv_ps[EWC];
    int inv_sn[EWC];
#pragma unroll
    for (int r = 0; r < EWC; ++r) {
        const int e = lane + 64 * r;
        const bool ok = e < E;
        if constexpr (PK == 1) {
            inv_ps[r] = ok ? ((uint32_t)pb.poss[e] | ((uint32_t)pb.sn[e] << 16)) : 0xFFFFu;
        } else {
            inv_poss[r] = ok ? (PossT)pb.poss[e] : (PossT)~0ull;
            inv_sn[r] = ok ? pb.sn[e] : 0;
        }
#pragma unroll
        for (int w = 0; w < EWC; ++w) inv_cup[r][w] = (w >= r && ok) ? pb.cupT[(size_t)w * E + e] : 0ull;
    }
    const ConstU32* rec = (const ConstU32*)pb.sch;
    const ConstI32* ptab = (const ConstI32*)pb.sch_part;
    const int pbase = NW == 4 ? kSchPart4 : kSchPart8;
    const int c0 = ptab[pbase + wv], c1 = ptab[pbase + wv + 1];
    const bool wide = (E & 15) == 0 && (((uintptr_t)slot) & 15) == 0;
    const int qpr = E >> 4;
    const uint32_t qinv = ((1u << 20) + (uint32_t)qpr - 1) / (uint32_t)max(qpr, 1);

    for (int tl = blockIdx.x; tl < tiles; tl += gridDim.x) {
        const long p0 = (long)tl * 64;
        const int np = (int)min((long)64, (long)P - p0);
        __syncthreads();
        // ---- stage the tile's slot rows (+ sentinel column E = slot 63)
        const uint8_t* src = slot + p0 * E;
        if (wide) {
            const uint4* s16 = (const uint4*)src;
#pragma unroll 2
            for (int w = threadIdx.x; w < np * qpr; w += NT) {
                const int r = (int)(((uint32_t)w * qinv) >> 20), c = w - r * qpr;
                const uint4 v = s16[w];
                uint32_t* d = (uint32_t*)(tile + r * SP + 16 * c);
                d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
            }
        } else {
#pragma unroll 1
            for (int r = wv; r < np; r += NW)
#pragma unroll 1
                for (int c = lane; c < E; c += 64) tile[r * SP + c] = src[(long)r * E + c];
        }
        if (threadIdx.x < 64) tile[threadIdx.x * SP + E] = 63;
        __syncthreads();

        // ---- lane phase (lane = individual): attendance masks of this wave's students
        int sc = 0;
        if (!(ablate & 1) && c0 < c1) {
            const uint8_t* my = tile + lane * SP;
            uint32_t cur[4] = {rec[4 * c0], rec[4 * c0 + 1], rec[4 * c0 + 2], rec[4 * c0 + 3]};
            uint64_t m = 0;
            for (int c = c0; c < c1; ++c) {
                const int cn = c + 1 < c1 ? c + 1 : c;
                const uint32_t nxt[4] = {rec[4 * cn], rec[4 * cn + 1], rec[4 * cn + 2], rec[4 * cn + 3]};
                uint32_t sl[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) sl[j] = my[(cur[j >> 1] >> (16 * (j & 1))) & 0x7FFFu];
#pragma unroll
                for (int j = 0; j < 8; ++j) m |= 1ull << (sl[j] & 63);
                if (cur[0] & 0x8000u) {                                  // last record of a student
                    sc += __popcll(m & (m >> 1) & (m >> 2) & kTripleMask);   // Solution.cpp:99-117
#pragma unroll
                    for (int d = 0; d < 5; ++d) sc += (__popc((uint32_t)(m >> (9 * d)) & 0x1FFu) == 1);   // :119-137
                    m = 0;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
            }
        }
        part[wv * 64 + lane] = sc;
        if constexpr (ALIAS) __syncthreads();                           // the tile is dead from here

        // ---- wave phase (wave = individual): hcv terms + last-slot term
        const int nq = (ablate & 2) ? 0 : np;
        // one row (slot rows if ALIAS, else room rows) is prefetched one individual ahead
        uint32_t pfn[EWC];
        auto load_row = [&](const uint8_t* base, int q, uint32_t* dst) {
            const uint8_t* rr = base + (p0 + q) * E;
#pragma unroll
            for (int r = 0; r < EWC; ++r)
                dst[r] = (!last_partial || r < EWC - 1 || lane + 64 * r < E) ? rr[lane + 64 * r] : 0u;
        };
        const uint8_t* pf_src = ALIAS ? slot : room;
        if (wv < nq) load_row(pf_src, wv, pfn);
        for (int q = wv; q < nq; q += NW) {
            uint32_t rv[EWC], sv[EWC];
            if constexpr (ALIAS) {
#pragma unroll
                for (int r = 0; r < EWC; ++r) sv[r] = pfn[r];
                load_row(room, q, rv);
            } else {
#pragma unroll
                for (int r = 0; r < EWC; ++r) rv[r] = pfn[r];
                const uint8_t* rs = tile + q * SP;
#pragma unroll
                for (int r = 0; r < EWC; ++r)
                    sv[r] = (!last_partial || r < EWC - 1 || lane + 64 * r < E) ? rs[lane + 64 * r] : 0u;
            }
            if (q + NW < nq) load_row(pf_src, q + NW, pfn);             // next individual
            // an invalid gene anywhere -> sentinel outputs; decided from registers
            uint32_t smax = 0, rmax = 0;
#pragma unroll
            for (int r = 0; r < EWC; ++r) { smax = max(smax, sv[r]); rmax = max(rmax, rv[r]); }
            const bool any_bad = __any(smax >= (uint32_t)kSlots || rmax >= (uint32_t)R);
            int h = 0, last = 0;
            if (!any_bad) {
                if (!(ablate & 32))
                    for (int c = lane; c < (L.WS >> 4); c += 64) ((uint4*)ws)[c] = make_uint4(0u, 0u, 0u, 0u);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int r = 0; r < EWC; ++r) {
                    if (r < EWC - 1 || !last_partial || lane + 64 * r < E) {
                        const uint32_t s = sv[r], ro = rv[r];
                        if (!(ablate & 8)) atomicOr((unsigned long long*)&B[s * EWC + r], 1ull << lane);
                        const uint32_t cell = s * (uint32_t)R + ro;
                        if (ablate & 16) {
                        } else if constexpr (CNT32) {
                            h += (int)atomicAdd(&cnt[cell], 1u);                        // Solution.cpp:148-150
                        } else {
                            const uint32_t sh = (cell & 1u) << 4;
                            h += (int)((atomicAdd(&cnt[cell >> 1], 1u << sh) >> sh) & 0xFFFFu);
                        }
                        const bool last_slot = (kLastSlotMask >> s) & 1ull;
                        if constexpr (PK == 1) {
                            h += (int)(((inv_ps[r] >> ro) & 1u) ^ 1u);                  // :155-156
                            last += last_slot ? (int)(inv_ps[r] >> 16) : 0;             // :93-96
                        } else {
                            h += (int)(((inv_poss[r] >> ro) & 1u) ^ 1u);
                            last += last_slot ? inv_sn[r] : 0;
                        }
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (!(ablate & 4)) {
                    // B-row words by single ds_read_b64 (2 LDS cycles per 512 B, 64 banks),
                    // not the ds_read2_b64 pairs the compiler forms (8 cycles per 1 KiB, 32 banks)
                    corr_words<0, EWC>(lds_addr(B), sv, inv_cup, lane, E, last_partial, h);   // :151-153
                }
                h = wave_sum(h);
                last = wave_sum(last);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            if (lane == 0) {
                hq[q] = any_bad ? -1 : h;
                part[wv * 64 + q] += last;
            }
        }
        __syncthreads();
        if (wv == 0 && lane < np) {
            const long p = p0 + lane;
            const int h = hq[lane];
            if (h < 0) {
                hcv_out[p] = -1; scv_out[p] = -1; feas_out[p] = 0; pen_out[p] = -1;
            } else {
                int s2 = 0;
#pragma unroll
                for (int w = 0; w < NW; ++w) s2 += part[w * 64 + lane];
                hcv_out[p] = h;
                scv_out[p] = s2;
                feas_out[p] = h == 0 ? 1 : 0;
                pen_out[p] = h == 0 ? s2 : 1000000 + h;
            }
        }
    }
}

// ---------------------------------------------------------------- eval_split
// The two phases of eval_tile5 as two launches on the same stream, so that
// each runs at the occupancy its own registers and LDS allow instead of the
// fused kernel's common minimum (128 VGPRs for the register-resident
// correlation words, a 26 KB tile per 64 individuals):
//  * eval_lanes_kernel (lane = individual): stages a tile, builds the
//    attendance masks of the wave's student range and writes the per-student
//    scv part (>2 in a row + single class) of each individual to scv_out;
//  * eval_waves_kernel (wave = individual, no tile, no workgroup barrier):
//    slot and room rows straight from global memory (one individual ahead),
//    the hcv terms and the last-slot term; it adds the latter to scv_out and
//    writes the final four outputs.
template <int NWL>
__global__ __launch_bounds__(64 * NWL) void eval_lanes_kernel(DevProblem pb, const uint8_t* __restrict__ slot, int P,
                                                              int32_t* __restrict__ scv_part) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int NT = 64 * NWL;
    const int E = pb.E;
    const int lane = threadIdx.x & 63, wv = wave_id();
    int sp = (E + 1 + 3) & ~3;
    if (((sp >> 2) & 1) == 0) sp += 4;
    const int SP = sp;
    uint8_t* tile = lds;
    int32_t* part = (int32_t*)(lds + (((size_t)64 * SP + 15) & ~(size_t)15));   // [NWL][64]
    const int tiles = (P + 63) / 64;
    const ConstU32* rec = (const ConstU32*)pb.sch;
    const ConstI32* ptab = (const ConstI32*)pb.sch_part;
    const int pbase = sch_part_base(NWL);
    const int c0 = ptab[pbase + wv], c1 = ptab[pbase + wv + 1];
    const bool wide = (E & 15) == 0 && (((uintptr_t)slot) & 15) == 0;
    const int qpr = E >> 4;
    const uint64_t qinv = ((1ull << 32) + (uint64_t)qpr - 1) / (uint64_t)max(qpr, 1);   // exact w / qpr below

    for (int tl = blockIdx.x; tl < tiles; tl += gridDim.x) {
        const long p0 = (long)tl * 64;
        const int np = (int)min((long)64, (long)P - p0);
        __syncthreads();
        const uint8_t* src = slot + p0 * E;
        if (wide) {
            const uint4* s16 = (const uint4*)src;
#pragma unroll 2
            for (int w = threadIdx.x; w < np * qpr; w += NT) {
                const int r = (int)(((uint64_t)(uint32_t)w * qinv) >> 32), c = w - r * qpr;
                const uint4 v = s16[w];
                uint32_t* d = (uint32_t*)(tile + r * SP + 16 * c);
                d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
            }
        } else {
#pragma unroll 1
            for (int r = wv; r < np; r += NWL)
#pragma unroll 1
                for (int c = lane; c < E; c += 64) tile[r * SP + c] = src[(long)r * E + c];
        }
        if (threadIdx.x < 64) tile[threadIdx.x * SP + E] = 63;
        __syncthreads();
        int sc = 0;
        if (c0 < c1) {
            const uint8_t* my = tile + lane * SP;
            uint32_t cur[4] = {rec[4 * c0], rec[4 * c0 + 1], rec[4 * c0 + 2], rec[4 * c0 + 3]};
            uint64_t m = 0;
            for (int c = c0; c < c1; ++c) {
                const int cn = c + 1 < c1 ? c + 1 : c;
                const uint32_t nxt[4] = {rec[4 * cn], rec[4 * cn + 1], rec[4 * cn + 2], rec[4 * cn + 3]};
                uint32_t sl[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) sl[j] = my[(cur[j >> 1] >> (16 * (j & 1))) & 0x7FFFu];
#pragma unroll
                for (int j = 0; j < 8; ++j) m |= 1ull << (sl[j] & 63);
                if (cur[0] & 0x8000u) {                                  // last record of a student
                    sc += __popcll(m & (m >> 1) & (m >> 2) & kTripleMask);   // Solution.cpp:99-117
#pragma unroll
                    for (int d = 0; d < 5; ++d) sc += (__popc((uint32_t)(m >> (9 * d)) & 0x1FFu) == 1);   // :119-137
                    m = 0;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) cur[k] = nxt[k];
            }
        }
        part[wv * 64 + lane] = sc;
        __syncthreads();
        if (wv == 0 && lane < np) {
            int s2 = 0;
#pragma unroll
            for (int w = 0; w < NWL; ++w) s2 += part[w * 64 + lane];
            scv_part[p0 + lane] = s2;
        }
    }
}

constexpr int kWavesWG = 4;   // waves per workgroup of eval_waves_kernel
constexpr int kWideWG = 8;    // waves per workgroup of eval_wide_kernel (one individual each)
constexpr int kWideMaxNC = 10; // eval_wide handles E <= 256 * kWideMaxNC

template <int EWC, int PK>
__global__ __launch_bounds__(64 * kWavesWG, 4) void eval_waves_kernel(DevProblem pb, const uint8_t* __restrict__ slot,
                                                                      const uint8_t* __restrict__ room, int P,
                                                                      int32_t* __restrict__ hcv_out,
                                                                      int32_t* __restrict__ scv_io,
                                                                      uint8_t* __restrict__ feas_out,
                                                                      int32_t* __restrict__ pen_out, int WS) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int E = pb.E, R = pb.R;
    const int lane = threadIdx.x & 63, wv = wave_id();
    uint8_t* ws = lds + (size_t)wv * WS;
    uint64_t* B = (uint64_t*)ws;                              // [45][EWC] event bitsets per slot
    uint32_t* cnt = (uint32_t*)(B + kSlots * EWC);            // packed u16 cell counters
    const bool last_partial = E < 64 * EWC;

    using PossT = typename std::conditional<PK == 0, uint64_t, uint32_t>::type;
    uint64_t inv_cup[EWC][EWC];
    PossT inv_poss[EWC];
    uint32_t inv_ps[EWC];
    int inv_sn[EWC];
#pragma unroll
    for (int r = 0; r < EWC; ++r) {
        const int e = lane + 64 * r;
        const bool ok = e < E;
        if constexpr (PK == 1) {
            inv_ps[r] = ok ? ((uint32_t)pb.poss[e] | ((uint32_t)pb.sn[e] << 16)) : 0xFFFFu;
        } else {
            inv_poss[r] = ok ? (PossT)pb.poss[e] : (PossT)~0ull;
            inv_sn[r] = ok ? pb.sn[e] : 0;
        }
#pragma unroll
        for (int w = 0; w < EWC; ++w) inv_cup[r][w] = (w >= r && ok) ? pb.cupT[(size_t)w * E + e] : 0ull;
    }
    auto load_row = [&](const uint8_t* base, long q, uint32_t* dst) {
        const uint8_t* rr = base + q * E;
#pragma unroll
        for (int r = 0; r < EWC; ++r)
            dst[r] = (!last_partial || r < EWC - 1 || lane + 64 * r < E) ? rr[lane + 64 * r] : 0u;
    };
    const long GW = (long)gridDim.x * kWavesWG;
    long q = (long)blockIdx.x * kWavesWG + wv;
    uint32_t svn[EWC], rvn[EWC];
    if (q < P) { load_row(slot, q, svn); load_row(room, q, rvn); }
    for (; q < P; q += GW) {
        uint32_t sv[EWC], rv[EWC];
#pragma unroll
        for (int r = 0; r < EWC; ++r) { sv[r] = svn[r]; rv[r] = rvn[r]; }
        if (q + GW < P) { load_row(slot, q + GW, svn); load_row(room, q + GW, rvn); }
        uint32_t smax = 0, rmax = 0;
#pragma unroll
        for (int r = 0; r < EWC; ++r) { smax = max(smax, sv[r]); rmax = max(rmax, rv[r]); }
        const bool any_bad = __any(smax >= (uint32_t)kSlots || rmax >= (uint32_t)R);
        int h = 0, last = 0;
        if (!any_bad) {
            for (int c = lane; c < (WS >> 4); c += 64) ((uint4*)ws)[c] = make_uint4(0u, 0u, 0u, 0u);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int r = 0; r < EWC; ++r) {
                if (r < EWC - 1 || !last_partial || lane + 64 * r < E) {
                    const uint32_t s = sv[r], ro = rv[r];
                    atomicOr((unsigned long long*)&B[s * EWC + r], 1ull << lane);
                    const uint32_t cell = s * (uint32_t)R + ro, sh = (cell & 1u) << 4;
                    h += (int)((atomicAdd(&cnt[cell >> 1], 1u << sh) >> sh) & 0xFFFFu);   // Solution.cpp:148-150
                    const bool last_slot = (kLastSlotMask >> s) & 1ull;
                    if constexpr (PK == 1) {
                        h += (int)(((inv_ps[r] >> ro) & 1u) ^ 1u);                  // :155-156
                        last += last_slot ? (int)(inv_ps[r] >> 16) : 0;             // :93-96
                    } else {
                        h += (int)(((inv_poss[r] >> ro) & 1u) ^ 1u);
                        last += last_slot ? inv_sn[r] : 0;
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            corr_words<0, EWC>(lds_addr(B), sv, inv_cup, lane, E, last_partial, h);   // :151-153
            h = wave_sum(h);
            last = wave_sum(last);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (lane == 0) {
            if (any_bad) {
                hcv_out[q] = -1; scv_io[q] = -1; feas_out[q] = 0; pen_out[q] = -1;
            } else {
                const int s2 = scv_io[q] + last;
                hcv_out[q] = h;
                scv_io[q] = s2;
                feas_out[q] = h == 0 ? 1 : 0;
                pen_out[q] = h == 0 ? s2 : 1000000 + h;
            }
        }
    }
}

// ---------------------------------------------------------------- eval_wide
// The wave phase for instances too wide for eval_tile5's register-resident
// correlation words (E > 448, e.g. the 2000-event synthetic instance), run
// after eval_lanes_kernel<16> (which writes the per-student scv part):
// wave = individual, NW waves (NW individuals) per workgroup, lane l owns
// events e = 256 c + 4 l + k (k < 4) of every 256-event chunk c < NC, so its
// slot/room bytes arrive as one dword per chunk and its invariants
// (possibleRooms, studentNumber, upper-triangle words) as 16-B vector loads.
// The upper-triangle words (E x EW64 / 2 u64, 256 KB at E = 2000) are the
// dominant stream: the waves of a workgroup walk them in the same order and
// meet at a barrier per chunk, so one wave's L2 fetch is the others' L1 hit.
// Per-wave LDS workspace: event bitsets B[45][BST] (BST = EW64 | 1 u64 words:
// an odd row stride spreads the 45 rows over the banks) and packed u16
// room-cell counters.
//   hcv  = sum over cells of C(n, 2)                (Solution.cpp:148-150, ds_add_rtn)
//        + sum_e [room_e not possible]              (:155-156)
//        + sum_e sum_{w >= e/64} popcount(cupT[w][e] & B[slot_e][w])   (:151-153)
//   scv += sum_e [slot_e % 9 == 8] studentNumber[e] (:93-96)
template <int NC, int NW>
__global__ __launch_bounds__(64 * NW) void eval_wide_kernel(DevProblem pb, const uint8_t* __restrict__ slot,
                                                            const uint8_t* __restrict__ room, int P,
                                                            int32_t* __restrict__ hcv_out,
                                                            int32_t* __restrict__ scv_io,
                                                            uint8_t* __restrict__ feas_out,
                                                            int32_t* __restrict__ pen_out, int BST, int WS,
                                                            int ablate) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int E = pb.E, R = pb.R, EW64 = pb.EW64;
    const int lane = threadIdx.x & 63, wv = wave_id();
    uint8_t* ws = lds + (size_t)wv * WS;
    uint64_t* B = (uint64_t*)ws;                              // [45][BST]
    uint32_t* cnt = (uint32_t*)(B + kSlots * BST);            // packed u16 cell counters
    // dword row loads and 16-B upper-triangle loads need E % 4 == 0 and aligned rows
    const bool al = (E & 3) == 0 && (((uintptr_t)slot | (uintptr_t)room) & 3) == 0;
    const int groups = (P + NW - 1) / NW;
    for (int g = blockIdx.x; g < groups; g += gridDim.x) {     // every wave runs every barrier
        const long q = (long)g * NW + wv;
        const bool act = q < P;
        uint32_t sv[NC], rv[NC];                              // bytes k = events 256c + 4 lane + k
        int nv[NC];                                           // valid events of the lane in chunk c
        bool bad = false;
        const uint8_t* srow = slot + (act ? q : 0) * E;
        const uint8_t* rrow = room + (act ? q : 0) * E;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int e0 = 256 * c + 4 * lane;
            nv[c] = act ? max(0, min(4, E - e0)) : 0;
            if (al && nv[c] == 4) {
                sv[c] = *(const uint32_t*)(srow + e0);
                rv[c] = *(const uint32_t*)(rrow + e0);
            } else {
                sv[c] = 0u; rv[c] = 0u;
                for (int k = 0; k < nv[c]; ++k) {
                    sv[c] |= (uint32_t)srow[e0 + k] << (8 * k);
                    rv[c] |= (uint32_t)rrow[e0 + k] << (8 * k);
                }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < nv[c]) bad |= ((sv[c] >> (8 * k)) & 0xFFu) >= (uint32_t)kSlots || ((rv[c] >> (8 * k)) & 0xFFu) >= (uint32_t)R;
        }
        const bool work = act && !__any(bad);                 // wave-uniform
        int h = 0, last = 0;
        if (work && !(ablate & 1)) {
            for (int i = lane; i < (WS >> 4); i += 64) ((uint4*)ws)[i] = make_uint4(0u, 0u, 0u, 0u);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int e0 = 256 * c + 4 * lane;
                if (nv[c] == 0) continue;
                uint64_t poss[4];
                int sn[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    poss[k] = k < nv[c] ? pb.poss[e0 + k] : ~0ull;
                    sn[k] = k < nv[c] ? pb.sn[e0 + k] : 0;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (k < nv[c]) {
                        const int e = e0 + k;
                        const uint32_t s = (sv[c] >> (8 * k)) & 0xFFu, ro = (rv[c] >> (8 * k)) & 0xFFu;
                        atomicOr((unsigned long long*)&B[s * (uint32_t)BST + (uint32_t)(e >> 6)], 1ull << (e & 63));
                        const uint32_t cell = s * (uint32_t)R + ro, sh = (cell & 1u) << 4;
                        h += (int)((atomicAdd(&cnt[cell >> 1], 1u << sh) >> sh) & 0xFFFFu);
                        h += (int)(((poss[k] >> ro) & 1ull) ^ 1ull);
                        last += ((kLastSlotMask >> s) & 1ull) ? sn[k] : 0;
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        // correlated same-slot pairs: the words w >= 4c hold every upper-triangle
        // bit of chunk c's events (bits j > e live in words >= e/64 >= 4c)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            __syncthreads();                                  // keep the group's waves on the same words
            const int e0 = 256 * c + 4 * lane;
            if (work && nv[c] > 0 && !(ablate & 2)) {
                uint32_t boff[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) boff[k] = ((sv[c] >> (8 * k)) & 0xFFu) * (uint32_t)BST;
                if (al) {                                     // nv[c] == 4; 32-B aligned words
#pragma unroll 4
                    for (int w = 4 * c; w < EW64; ++w) {
                        const uint4* cw = (const uint4*)(pb.cupT + (size_t)w * E + e0);
                        const uint4 x = cw[0], y = cw[1];
                        h += __popcll((((uint64_t)x.y << 32) | x.x) & B[boff[0] + (uint32_t)w]);
                        h += __popcll((((uint64_t)x.w << 32) | x.z) & B[boff[1] + (uint32_t)w]);
                        h += __popcll((((uint64_t)y.y << 32) | y.x) & B[boff[2] + (uint32_t)w]);
                        h += __popcll((((uint64_t)y.w << 32) | y.z) & B[boff[3] + (uint32_t)w]);
                    }
                } else {
#pragma unroll 2
                    for (int w = 4 * c; w < EW64; ++w) {
                        const uint64_t* cw = pb.cupT + (size_t)w * E + e0;
#pragma unroll
                        for (int k = 0; k < 4; ++k)
                            if (k < nv[c]) h += __popcll(cw[k] & B[boff[k] + (uint32_t)w]);
                    }
                }
            }
        }
        if (work) {
            h = wave_sum(h);
            last = wave_sum(last);
        }
        if (act && lane == 0) {
            if (!work) {
                hcv_out[q] = -1; scv_io[q] = -1; feas_out[q] = 0; pen_out[q] = -1;
            } else {
                const int s2 = scv_io[q] + last;
                hcv_out[q] = h;
                scv_io[q] = s2;
                feas_out[q] = h == 0 ? 1 : 0;
                pen_out[q] = h == 0 ? s2 : 1000000 + h;
            }
        }
        __syncthreads();                                      // workspaces are reused by the next group
    }
}

struct WideLayout {
    int BST, WS;
    size_t lanes_bytes;
};

// LDS of the wide path: eval_lanes_kernel<16> tile + partials, per-wave workspace of eval_wide_kernel.
static WideLayout wide_layout(int E, int R, int EW64) {
    WideLayout L;
    L.BST = EW64 | 1;
    L.WS = (kSlots * L.BST * 8 + ((kSlots * R + 1) / 2) * 4 + 15) & ~15;
    int sp = (E + 1 + 3) & ~3;
    if (((sp >> 2) & 1) == 0) sp += 4;
    L.lanes_bytes = (((size_t)64 * sp + 15) & ~(size_t)15) + 4 * (size_t)16 * 64;
    return L;
}

// ---------------------------------------------------------------- eval_block
constexpr int kBlockThreads = 256;

__global__ __launch_bounds__(kBlockThreads) void eval_block_kernel(DevProblem pb, const uint8_t* __restrict__ slot,
                                                                   const uint8_t* __restrict__ room, int P,
                                                                   int32_t* __restrict__ hcv_out,
                                                                   int32_t* __restrict__ scv_out,
                                                                   uint8_t* __restrict__ feas_out,
                                                                   int32_t* __restrict__ pen_out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int E = pb.E, R = pb.R, S = pb.S, EW = pb.EW;
    const int tid = threadIdx.x;
    const long p = blockIdx.x;
    const int cells = kSlots * R;
    uint32_t* cnt = (uint32_t*)lds;                       // [cells]
    uint32_t* bcnt = cnt + cells;                         // [45] events per slot
    uint32_t* bstart = bcnt + kSlots;                     // [45]
    uint32_t* bcur = bstart + kSlots;                     // [45]
    int32_t* red = (int32_t*)(bcur + kSlots);             // [4] hcv, scv, bad
    uint16_t* bucket = (uint16_t*)(red + 4);              // [E]
    uint8_t* sl = (uint8_t*)(bucket + ((E + 1) & ~1));    // [E]

    const uint8_t* gs = slot + p * E;
    const uint8_t* gr = room + p * E;
    for (int c = tid; c < cells; c += kBlockThreads) cnt[c] = 0u;
    for (int c = tid; c < kSlots; c += kBlockThreads) { bcnt[c] = 0u; bcur[c] = 0u; }
    if (tid < 4) red[tid] = 0;
    for (int e = tid; e < E; e += kBlockThreads) sl[e] = gs[e];
    __syncthreads();

    int h = 0, sc = 0;
    bool bad = false;
    for (int e = tid; e < E; e += kBlockThreads) {
        const int s = sl[e], r = gr[e];
        if (s >= kSlots || r >= R) { bad = true; continue; }
        h += (int)atomicAdd(&cnt[s * R + r], 1u);
        h += ((pb.poss[e] >> r) & 1ull) ? 0 : 1;
        sc += ((kLastSlotMask >> s) & 1ull) ? pb.sn[e] : 0;
        atomicAdd(&bcnt[s], 1u);
    }
    if (bad) atomicOr(&red[2], 1);
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        for (int t = 0; t < kSlots; ++t) { bstart[t] = acc; acc += bcnt[t]; }
    }
    __syncthreads();
    if (red[2] == 0) {
        for (int e = tid; e < E; e += kBlockThreads) {
            const int s = sl[e];
            bucket[bstart[s] + atomicAdd(&bcur[s], 1u)] = (uint16_t)e;
        }
    }
    __syncthreads();
    if (red[2] == 0) {
        // correlated same-slot pairs, enumerated inside each slot's bucket
        for (int i = tid; i < E; i += kBlockThreads) {
            const int s = sl[i];
            const uint32_t* row = pb.corr + (size_t)i * EW;
            const uint32_t b0 = bstart[s], b1 = b0 + bcnt[s];
            for (uint32_t b = b0; b < b1; ++b) {
                const int j = bucket[b];
                if (j > i) h += (row[j >> 5] >> (j & 31)) & 1u;
            }
        }
        // per-student masks
        for (int st = tid; st < S; st += kBlockThreads) {
            uint64_t m = 0;
            for (int k = pb.stu_off[st]; k < pb.stu_off[st + 1]; ++k) m |= 1ull << sl[pb.stu_ev[k]];
            sc += __popcll(m & (m >> 1) & (m >> 2) & kTripleMask);
#pragma unroll
            for (int d = 0; d < 5; ++d) sc += (__popc((uint32_t)(m >> (9 * d)) & 0x1FFu) == 1);
        }
    }
    h = wave_sum(h);
    sc = wave_sum(sc);
    if ((tid & 63) == 0) { atomicAdd(&red[0], h); atomicAdd(&red[1], sc); }
    __syncthreads();
    if (tid == 0) {
        if (red[2]) {
            hcv_out[p] = -1; scv_out[p] = -1; feas_out[p] = 0; pen_out[p] = -1;
        } else {
            const int hh = red[0], ss = red[1];
            hcv_out[p] = hh;
            scv_out[p] = ss;
            feas_out[p] = hh == 0 ? 1 : 0;
            pen_out[p] = hh == 0 ? ss : 1000000 + hh;
        }
    }
}

static size_t block_lds_bytes(int E, int R) {
    return 4 * (size_t)(kSlots * R + 3 * kSlots + 4) + 2 * (size_t)((E + 1) & ~1) + (size_t)E;
}

}  // namespace ttga

using namespace ttga;

// The kernel tt_eval runs for this instance (see tt_eval_variant).
static int auto_variant(const tt_problem* p) {
    const int E = p->E, R = p->R;
    if (p->dev.EW64 <= 7 && E <= 32767 && tile5_layout(E, R, 8, false, false).bytes <= 80 * 1024) return 8;
    if (p->dev.EW64 <= 7 && tile4_layout(E, R, 4).bytes <= 64 * 1024) return 3;
    const WideLayout WL = wide_layout(E, R, p->dev.EW64);
    if (E <= 256 * kWideMaxNC && E <= 32767 && WL.lanes_bytes <= 160 * 1024 && (size_t)(kWideWG / 2) * WL.WS <= 160 * 1024)
        return 13;
    return (E <= 1024 && tile_layout(E, R).bytes <= 80 * 1024) ? 1 : 2;
}

extern "C" int tt_eval_auto_variant(const tt_problem* p) { return p ? auto_variant(p) : -1; }

extern "C" int tt_eval_variant(const tt_problem* p, const uint8_t* slot, const uint8_t* room, int P, int32_t* hcv,
                               int32_t* scv, uint8_t* feasible, int32_t* penalty, int variant, void* stream) {
    int rc = check_pop_args(p, P, slot, room);
    if (rc) return rc;
    if (P > 0 && (!hcv || !scv || !feasible || !penalty)) { set_error("null output buffer"); return TT_ERR_INVALID; }
    // profiling-only phase switches (results invalid): 1 lane phase, 2 wave phase, 4 correlation
    // words, 8 B-bitset atomics, 16 cell-counter atomics, 32 workspace zeroing (eval_tile5);
    // 1 atomics + zeroing, 2 correlation words (eval_wide)
    const int ablate = variant >> 4;
    variant &= 15;
    if (variant < 0 || variant > 13) { set_error("unknown eval variant"); return TT_ERR_INVALID; }
    if (P == 0) return TT_OK;
    rc = use_device(p);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int E = p->E, R = p->R;
    const TileLayout TL = tile_layout(E, R);
    if (variant == 0) variant = auto_variant(p);
    if (variant == 1) {
        if (TL.bytes > 160 * 1024) { set_error("instance too large for the tile kernel"); return TT_ERR_LIMIT; }
        const int tiles = (P + 63) / 64;
        const dim3 b(64 * kTileWaves);
        auto launch = [&](auto kern) -> int {
            int per_cu = 0;
            TT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, b.x, TL.bytes));
            const int grid = std::min(tiles, std::max(1, per_cu) * p->num_cus);
            hipLaunchKernelGGL(kern, dim3(grid), b, TL.bytes, st, p->dev, slot, room, P, hcv, scv, feasible, penalty,
                               ablate);
            return TT_OK;
        };
        switch (p->dev.EW64) {
            case 1: rc = launch(eval_tile_kernel<1>); break;
            case 2: rc = launch(eval_tile_kernel<2>); break;
            case 3: rc = launch(eval_tile_kernel<3>); break;
            case 4: rc = launch(eval_tile_kernel<4>); break;
            case 5: rc = launch(eval_tile_kernel<5>); break;
            case 6: rc = launch(eval_tile_kernel<6>); break;
            case 7: rc = launch(eval_tile_kernel<7>); break;
            default: rc = launch(eval_tile_kernel<0>); break;
        }
        if (rc) return rc;
    } else if (variant == 3 || variant == 4) {
        const int NW = variant == 3 ? 4 : 8;
        const Tile4Layout TL4 = tile4_layout(E, R, NW);
        if (p->dev.EW64 > 7 || TL4.bytes > 160 * 1024) { set_error("instance too large for the tile4 kernel"); return TT_ERR_LIMIT; }
        const int max_sn = p->student_number.empty() ? 0 : *std::max_element(p->student_number.begin(), p->student_number.end());
        const int pk = (R <= 16 && max_sn <= 0xFFFF) ? 1 : R <= 32 ? 2 : 0;
        const int tiles = (P + 63) / 64;
        auto launch = [&](auto kern) -> int {
            int per_cu = 0;
            TT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * NW, TL4.bytes));
            const int grid = std::min(tiles, std::max(1, per_cu) * p->num_cus);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * NW), TL4.bytes, st, p->dev, slot, room, P, hcv, scv,
                               feasible, penalty, ablate);
            return TT_OK;
        };
#define TT_T4(EWC)                                                                              \
    case EWC:                                                                                   \
        if (NW == 4) rc = pk == 1 ? launch(eval_tile4_kernel<EWC, 4, 1>) : pk == 2 ? launch(eval_tile4_kernel<EWC, 4, 2>) \
                                  : launch(eval_tile4_kernel<EWC, 4, 0>);                                         \
        else rc = pk == 1 ? launch(eval_tile4_kernel<EWC, 8, 1>) : pk == 2 ? launch(eval_tile4_kernel<EWC, 8, 2>)     \
                          : launch(eval_tile4_kernel<EWC, 8, 0>);                                                 \
        break;
        switch (p->dev.EW64) {
            TT_T4(1) TT_T4(2) TT_T4(3) TT_T4(4) TT_T4(5) TT_T4(6) TT_T4(7)
            default: rc = TT_ERR_LIMIT; break;
        }
#undef TT_T4
        if (rc) return rc;
    } else if (variant == 9 || variant == 10) {
        // eval_lanes (8 or 4 waves per tile) then eval_waves, both on `st`
        if (p->dev.EW64 > 7 || E > 32767) { set_error("instance too large for the split kernels"); return TT_ERR_LIMIT; }
        const int NWL = variant == 9 ? 8 : 4;
        int sp = (E + 1 + 3) & ~3;
        if (((sp >> 2) & 1) == 0) sp += 4;
        const size_t lds_l = (((size_t)64 * sp + 15) & ~(size_t)15) + 4 * (size_t)NWL * 64;
        const int tiles = (P + 63) / 64;
        auto launch_l = [&](auto kern) -> int {
            int per_cu = 0;
            TT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * NWL, lds_l));
            const int grid = std::min(tiles, std::max(1, per_cu) * p->num_cus);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * NWL), lds_l, st, p->dev, slot, P, scv);
            return TT_OK;
        };
        rc = NWL == 8 ? launch_l(eval_lanes_kernel<8>) : launch_l(eval_lanes_kernel<4>);
        if (rc) return rc;
        const int WS = tile5_layout(E, R, 8, false, false).WS;
        const size_t lds_w = (size_t)kWavesWG * WS;
        const int max_sn = p->student_number.empty() ? 0 : *std::max_element(p->student_number.begin(), p->student_number.end());
        const int pk = (R <= 16 && max_sn <= 0xFFFF) ? 1 : R <= 32 ? 2 : 0;
        auto launch_w = [&](auto kern) -> int {
            int per_cu = 0;
            TT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * kWavesWG, lds_w));
            const int grid = std::min((P + kWavesWG - 1) / kWavesWG, std::max(1, per_cu) * p->num_cus);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * kWavesWG), lds_w, st, p->dev, slot, room, P, hcv, scv,
                               feasible, penalty, WS);
            return TT_OK;
        };
#define TT_TW(EWC)                                                                                  \
    case EWC:                                                                                       \
        rc = pk == 1 ? launch_w(eval_waves_kernel<EWC, 1>) : pk == 2 ? launch_w(eval_waves_kernel<EWC, 2>) \
                     : launch_w(eval_waves_kernel<EWC, 0>);                                          \
        break;
        switch (p->dev.EW64) {
            TT_TW(1) TT_TW(2) TT_TW(3) TT_TW(4) TT_TW(5) TT_TW(6) TT_TW(7)
            default: rc = TT_ERR_LIMIT; break;
        }
#undef TT_TW
        if (rc) return rc;
    } else if (variant == 13) {
        // wide path: eval_lanes<16> (tile of 64 rows, lane phase) then eval_wide (wave = individual)
        const WideLayout WL = wide_layout(E, R, p->dev.EW64);
        if (E > 256 * kWideMaxNC || E > 32767 || WL.lanes_bytes > 160 * 1024 || (size_t)(kWideWG / 2) * WL.WS > 160 * 1024) {
            set_error("instance outside the wide eval path");
            return TT_ERR_LIMIT;
        }
        const int tiles = (P + 63) / 64;
        {
            int per_cu = 0;
            TT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, eval_lanes_kernel<16>, 1024, WL.lanes_bytes));
            const int grid = std::min(tiles, std::max(1, per_cu) * p->num_cus);
            hipLaunchKernelGGL(eval_lanes_kernel<16>, dim3(grid), dim3(1024), WL.lanes_bytes, st, p->dev, slot, P, scv);
        }
        // 8 individuals per workgroup, or 4 where 8 workspaces exceed the LDS
        const int NWW = (size_t)kWideWG * WL.WS <= 160 * 1024 ? kWideWG : kWideWG / 2;
        const size_t lds_w = (size_t)NWW * WL.WS;
        auto launch_w = [&](auto kern) -> int {
            int per_cu = 0;
            TT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * NWW, lds_w));
            const int grid = (int)std::min<long>(((long)P + NWW - 1) / NWW, (long)std::max(1, per_cu) * p->num_cus);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * NWW), lds_w, st, p->dev, slot, room, P, hcv, scv,
                               feasible, penalty, WL.BST, WL.WS, ablate);
            return TT_OK;
        };
#define TT_WD(NC) \
    case NC: rc = NWW == kWideWG ? launch_w(eval_wide_kernel<NC, kWideWG>) : launch_w(eval_wide_kernel<NC, kWideWG / 2>); break;
        switch ((E + 255) / 256) {
            TT_WD(1) TT_WD(2) TT_WD(3) TT_WD(4) TT_WD(5) TT_WD(6) TT_WD(7) TT_WD(8) TT_WD(9) TT_WD(10)
            default: rc = TT_ERR_LIMIT; break;
        }
#undef TT_WD
        if (rc) return rc;
    } else if (variant >= 5 && variant <= 8) {
        // 5/6: eval_tile5 with 4/8 waves, workspaces aliased on the tile, u32 cell
        // counters; 7/8: tile kept for the wave phase, packed u16 counters
        const int NW = (variant == 5 || variant == 7) ? 4 : 8;
        const bool c32 = variant <= 6;          // u32 counters live on top of the dead tile
        const Tile5Layout TL5 = tile5_layout(E, R, NW, c32, c32);
        if (p->dev.EW64 > 7 || TL5.bytes > 160 * 1024 || E > 32767) {
            set_error("instance too large for the tile5 kernel");
            return TT_ERR_LIMIT;
        }
        const int max_sn = p->student_number.empty() ? 0 : *std::max_element(p->student_number.begin(), p->student_number.end());
        const int pk = (R <= 16 && max_sn <= 0xFFFF) ? 1 : R <= 32 ? 2 : 0;
        const int tiles = (P + 63) / 64;
        auto launch = [&](auto kern) -> int {
            int per_cu = 0;
            TT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * NW, TL5.bytes));
            const int grid = std::min(tiles, std::max(1, per_cu) * p->num_cus);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * NW), TL5.bytes, st, p->dev, slot, room, P, hcv, scv,
                               feasible, penalty, ablate);
            return TT_OK;
        };
#define TT_T5N(EWC, NWV, C)                                                                          \
    rc = pk == 1 ? launch(eval_tile5_kernel<EWC, NWV, C, 1, C>) : pk == 2 ? launch(eval_tile5_kernel<EWC, NWV, C, 2, C>) \
                 : launch(eval_tile5_kernel<EWC, NWV, C, 0, C>);
#define TT_T5(EWC)                                                      \
    case EWC:                                                           \
        if (NW == 4) { if (c32) { TT_T5N(EWC, 4, true) } else { TT_T5N(EWC, 4, false) } } \
        else { if (c32) { TT_T5N(EWC, 8, true) } else { TT_T5N(EWC, 8, false) } }         \
        break;
        switch (p->dev.EW64) {
            TT_T5(1) TT_T5(2) TT_T5(3) TT_T5(4) TT_T5(5) TT_T5(6) TT_T5(7)
            default: rc = TT_ERR_LIMIT; break;
        }
#undef TT_T5
#undef TT_T5N
        if (rc) return rc;
    } else {
        const size_t lds = block_lds_bytes(E, R);
        if (lds > 160 * 1024) { set_error("instance too large for the block kernel"); return TT_ERR_LIMIT; }
        hipLaunchKernelGGL(eval_block_kernel, dim3(P), dim3(kBlockThreads), lds, st, p->dev, slot, room, P, hcv,
                           scv, feasible, penalty);
    }
    return check_hip(hipGetLastError(), "tt_eval launch");
}

extern "C" int tt_eval(const tt_problem* p, const uint8_t* slot, const uint8_t* room, int P, int32_t* hcv,
                       int32_t* scv, uint8_t* feasible, int32_t* penalty, void* stream) {
    return tt_eval_variant(p, slot, room, P, hcv, scv, feasible, penalty, 0, stream);
}

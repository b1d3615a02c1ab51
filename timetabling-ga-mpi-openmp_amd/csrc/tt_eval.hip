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
//  * eval_lanes (E <= 1024): one wave per 64 individuals. The individuals'
//    slot rows are staged in LDS with an odd-dword row stride; the per-student
//    attendance masks, the last-slot term and the correlated-pair term run
//    LANE = INDIVIDUAL with wave-uniform loops over the problem's sparse
//    structure (scalar loads, no divergence, conflict-free ds_read_u8); the
//    room-clash term runs WAVE = INDIVIDUAL with LDS atomic cell counters.
//  * eval_block (any E): one 256-thread workgroup per individual; slot
//    buckets in LDS enumerate only same-slot pairs for the correlation term.
#include "tt_internal.h"

namespace ttga {

// ---------------------------------------------------------------- eval_lanes
__global__ __launch_bounds__(64) void eval_lanes_kernel(DevProblem pb, const uint8_t* __restrict__ slot,
                                                        const uint8_t* __restrict__ room, int P, int SP,
                                                        int32_t* __restrict__ hcv_out, int32_t* __restrict__ scv_out,
                                                        uint8_t* __restrict__ feas_out, int32_t* __restrict__ pen_out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int E = pb.E, R = pb.R, S = pb.S;
    const int lane = threadIdx.x;
    const long p0 = (long)blockIdx.x * 64;
    const int np = (int)min((long)64, (long)P - p0);
    uint8_t* tile = lds;                                           // [64][SP] slot rows
    uint32_t* cnt = (uint32_t*)(lds + 64 * SP);                    // [45*R] cell counters
    int32_t* xfer = (int32_t*)(cnt + ((kSlots * R + 3) & ~3));     // [64] room-term per individual

    // ---- stage the slot rows of this wave's individuals into LDS
    const uint8_t* src = slot + p0 * E;
    if ((E & 3) == 0) {
        const int wpr = E >> 2;
        const uint32_t* s32 = (const uint32_t*)src;
        const int nw = np * wpr;
        for (int w = lane; w < nw; w += 64) {
            int r = w / wpr, c = w - r * wpr;
            *(uint32_t*)(tile + r * SP + 4 * c) = s32[w];
        }
    } else {
        const int nb = np * E;
        for (int b = lane; b < nb; b += 64) {
            int r = b / E, c = b - r * E;
            tile[r * SP + c] = src[b];
        }
    }
    __syncthreads();

    // ---- lane = individual (lanes >= np read a stale row; their results are dropped)
    const uint8_t* my = tile + lane * SP;
    int last = 0, cons = 0, single = 0, corr = 0;

    // last slot of the day: Solution.cpp:93-96
#pragma unroll 4
    for (int e = 0; e < E; ++e) {
        int s = my[e];
        last += ((kLastSlotMask >> s) & 1ull) ? pb.sn[e] : 0;
    }

    // per-student attendance masks: Solution.cpp:98-137
    for (int st = 0; st < S; ++st) {
        const int k0 = pb.stu_off[st], k1 = pb.stu_off[st + 1];
        uint64_t m = 0;
        for (int k = k0; k < k1; ++k) m |= 1ull << my[pb.stu_ev[k]];
        cons += __popcll(m & (m >> 1) & (m >> 2) & kTripleMask);
#pragma unroll
        for (int d = 0; d < 5; ++d) {
            uint32_t f = (uint32_t)(m >> (9 * d)) & 0x1FFu;
            single += (__popc(f) == 1);
        }
    }

    // correlated events in one slot: Solution.cpp:151-153
    for (int i = 0; i < E; ++i) {
        const int k0 = pb.cp_off[i], k1 = pb.cp_off[i + 1];
        if (k0 == k1) continue;
        const int si = my[i];
        int c = 0;
#pragma unroll 4
        for (int k = k0; k < k1; ++k) c += (my[pb.cp_j[k]] == si);
        corr += c;
    }

    // ---- wave = individual: room clashes (Solution.cpp:148-150) and unsuitable rooms (:155-156)
    const int cells = kSlots * R;
    for (int q = 0; q < np; ++q) {
        for (int c = lane; c < cells; c += 64) cnt[c] = 0u;
        __syncthreads();
        const uint8_t* rs = tile + q * SP;
        const uint8_t* rr = room + (p0 + q) * E;
        int acc = 0;
        bool bad = false;
        for (int e = lane; e < E; e += 64) {
            const int s = rs[e], r = rr[e];
            if (s >= kSlots || r >= R) { bad = true; continue; }
            acc += (int)atomicAdd(&cnt[s * R + r], 1u);
            acc += ((pb.poss[e] >> r) & 1ull) ? 0 : 1;
        }
        acc = wave_sum(acc);
        const bool any_bad = __any(bad);
        if (lane == 0) xfer[q] = any_bad ? -1 : acc;
        __syncthreads();
    }

    if (lane < np) {
        const long p = p0 + lane;
        const int rt = xfer[lane];
        if (rt < 0) {
            hcv_out[p] = -1; scv_out[p] = -1; feas_out[p] = 0; pen_out[p] = -1;
        } else {
            const int h = rt + corr;
            const int sc = last + cons + single;
            hcv_out[p] = h;
            scv_out[p] = sc;
            feas_out[p] = h == 0 ? 1 : 0;
            pen_out[p] = h == 0 ? sc : 1000000 + h;
        }
    }
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

static int lane_stride(int E) {
    int sp = (E + 3) & ~3;           // dword-aligned rows
    if (((sp >> 2) & 1) == 0) sp += 4;  // odd dword count: conflict-free column reads
    return sp;
}

static size_t lanes_lds_bytes(int E, int R) {
    return (size_t)64 * lane_stride(E) + 4 * (size_t)((kSlots * R + 3) & ~3) + 64 * 4;
}

static size_t block_lds_bytes(int E, int R) {
    return 4 * (size_t)(kSlots * R + 3 * kSlots + 4) + 2 * (size_t)((E + 1) & ~1) + (size_t)E;
}

}  // namespace ttga

using namespace ttga;

extern "C" int tt_eval_variant(const tt_problem* p, const uint8_t* slot, const uint8_t* room, int P, int32_t* hcv,
                               int32_t* scv, uint8_t* feasible, int32_t* penalty, int variant, void* stream) {
    int rc = check_pop_args(p, P, slot, room);
    if (rc) return rc;
    if (P > 0 && (!hcv || !scv || !feasible || !penalty)) { set_error("null output buffer"); return TT_ERR_INVALID; }
    if (variant < 0 || variant > 2) { set_error("unknown eval variant"); return TT_ERR_INVALID; }
    if (P == 0) return TT_OK;
    rc = use_device(p);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int E = p->E, R = p->R;
    const size_t lanes_lds = lanes_lds_bytes(E, R);
    if (variant == 0) variant = (E <= 1024 && lanes_lds <= 65536) ? 1 : 2;
    if (variant == 1) {
        if (lanes_lds > 160 * 1024) { set_error("instance too large for the lane kernel"); return TT_ERR_LIMIT; }
        const int blocks = (P + 63) / 64;
        hipLaunchKernelGGL(eval_lanes_kernel, dim3(blocks), dim3(64), lanes_lds, st, p->dev, slot, room, P,
                           lane_stride(E), hcv, scv, feasible, penalty);
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

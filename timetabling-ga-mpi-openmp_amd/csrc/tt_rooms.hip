// Room assignment and the variation operators that end in it:
//   tt_assign_rooms  Solution::assignRooms on every non-empty slot (Solution.cpp:772-891)
//   tt_random_init   Solution::RandomInitialSolution        (Solution.cpp:48-61)
//   tt_crossover     Solution::crossover on a fresh child   (Solution.cpp:893-910)
//   tt_mutation      Solution::mutation -> randomMove       (Solution.cpp:441-469,912-914)
#include "tt_internal.h"
#include "tt_match.h"

namespace ttga {

constexpr int kMaxRejections = 1 << 20;
#ifndef TT_ROOMS_ABL
#define TT_ROOMS_ABL 0
#endif

// ---------------------------------------------------------------- helpers
// 512 bytes per block: the block's eight loads are all in flight before the
// first LDS store (a plain loop waits out one HBM latency per 64 bytes)
__device__ inline void load_row(uint8_t* dst, const uint8_t* src, int E, int lane) {
    for (int e0 = 0; e0 < E; e0 += 512) {
        uint8_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int e = e0 + 64 * k + lane;
            v[k] = e < E ? src[e] : 0;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int e = e0 + 64 * k + lane;
            if (e < E) dst[e] = v[k];
        }
    }
}

__device__ inline void store_row(uint8_t* dst, const uint8_t* src, int E, int lane) {
    for (int e = lane; e < E; e += 64) dst[e] = src[e];
}

// ---------------------------------------------------------------- assign
// One individual per workgroup of 64 threads, or (wide layout, R > 16) of
// kWideWaves waves: the first loads the row and builds the buckets, then the
// waves match alternate slots (their searches are long; a shared individual
// halves the LDS per wave, so twice as many waves hide each other's latency).
__global__ __launch_bounds__(64 * kWideWaves) void assign_rooms_kernel(DevProblem pb, const uint8_t* __restrict__ slot,
                                                                       uint8_t* __restrict__ room, int P,
                                                                       const uint8_t* __restrict__ mask, uint8_t bit) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int E = pb.E, lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const long p = blockIdx.x;
    if (mask && !(mask[p] & bit)) return;
    MatchScratch m = carve_match_scratch(lds, E, pb.R, nw);
    if (w == 0) {
        load_row(m.sl, slot + p * E, E, lane);
        for (int e = lane; e < E; e += 64) m.rr[e] = 0xFF;   // events with an invalid slot stay 255
    }
    __syncthreads();
    build_buckets(pb, m, lane, w == 0);
#if TT_ROOMS_ABL != 1                                    // profiling builds only: buckets alone
    assign_touched(pb, m, ~0ull, lane, w, nw);
#endif
    if (w == 0) store_row(room + p * E, m.rr, E, lane);
}

// ---------------------------------------------------------------- lane-per-individual slot generators
// Rows of 64 individuals are built in LDS (row stride SP) and written out
// coalesced; RNG streams advance exactly as the reference's per-event draws.
__device__ inline void flush_tile(uint8_t* dst, const uint8_t* tile, int SP, int E, int np, int lane) {
    const int nb = np * E;
    for (int b = lane; b < nb; b += 64) {
        const int r = b / E, c = b - r * E;
        dst[b] = tile[r * SP + c];
    }
}

__device__ inline void fill_tile(uint8_t* tile, const uint8_t* src, int SP, int E, int np, int lane) {
    const int nb = np * E;
    for (int b = lane; b < nb; b += 64) {
        const int r = b / E, c = b - r * E;
        tile[r * SP + c] = src[b];
    }
}

__global__ __launch_bounds__(64) void rand_slots_kernel(int E, int64_t* __restrict__ rng, uint8_t* __restrict__ slot,
                                                        int P, int SP) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x;
    const long p0 = (long)blockIdx.x * 64;
    const int np = (int)min((long)64, (long)P - p0);
    if (lane < np) {
        int64_t s = rng[p0 + lane];
        uint8_t* row = lds + lane * SP;
        for (int e = 0; e < E; ++e) row[e] = (uint8_t)pm_pick(s, kSlots);   // Solution.cpp:52
        rng[p0 + lane] = s;
    }
    __syncthreads();
    flush_tile(slot + p0 * E, lds, SP, E, np, lane);
}

__global__ __launch_bounds__(64) void crossover_slots_kernel(int E, const uint8_t* __restrict__ s1,
                                                             const uint8_t* __restrict__ s2,
                                                             int64_t* __restrict__ rng, uint8_t* __restrict__ child,
                                                             int P, int SP) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x;
    const long p0 = (long)blockIdx.x * 64;
    const int np = (int)min((long)64, (long)P - p0);
    uint8_t* t1 = lds;
    uint8_t* t2 = lds + 64 * SP;
    fill_tile(t1, s1 + p0 * E, SP, E, np, lane);
    fill_tile(t2, s2 + p0 * E, SP, E, np, lane);
    __syncthreads();
    if (lane < np) {
        int64_t s = rng[p0 + lane];
        uint8_t* a = t1 + lane * SP;
        const uint8_t* b = t2 + lane * SP;
        for (int e = 0; e < E; ++e)                                      // Solution.cpp:896-903
            if (!(pm_next(s) < 0.5)) a[e] = b[e];
        rng[p0 + lane] = s;
    }
    __syncthreads();
    flush_tile(child + p0 * E, t1, SP, E, np, lane);
}

// ---------------------------------------------------------------- mutation
// One wave per individual: lane 0 replays randomMove's draws (Solution.cpp:441-469)
// and the slot changes of Move1/2/3 (:357-439); the wave then re-assigns the
// touched slots (the reference re-runs assignRooms on each of them; a slot
// touched twice gets the same rooms both times).
__global__ __launch_bounds__(64) void mutation_kernel(DevProblem pb, uint8_t* __restrict__ slot,
                                                      uint8_t* __restrict__ room, int64_t* __restrict__ rng,
                                                      int P, const uint8_t* __restrict__ mask, uint8_t bit) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int E = pb.E, lane = threadIdx.x;
    const long p = blockIdx.x;
    if (mask && !(mask[p] & bit)) return;
    MatchScratch m = carve_match_scratch(lds, E, pb.R);
    load_row(m.sl, slot + p * E, E, lane);
    load_row(m.rr, room + p * E, E, lane);
    __syncthreads();
    if (lane == 0) {
        int64_t s = rng[p];
        uint64_t touched = 0;
        const int type = pm_pick(s, 3) + 1;
        const int e1 = pm_pick(s, E);
        if (type == 1) {
            const int t = pm_pick(s, kSlots);
            touched = (1ull << t) | (1ull << m.sl[e1]);
            m.sl[e1] = (uint8_t)t;
        } else if (type == 2) {
            // the reference's rejection loops never end for E < 2 / E < 3; bound them
            int e2 = pm_pick(s, E);
            for (int g = 0; e2 == e1 && g < kMaxRejections; ++g) e2 = pm_pick(s, E);
            const uint8_t t = m.sl[e1];
            touched = (1ull << t) | (1ull << m.sl[e2]);
            m.sl[e1] = m.sl[e2];
            m.sl[e2] = t;
        } else {
            int e2 = pm_pick(s, E);
            for (int g = 0; e2 == e1 && g < kMaxRejections; ++g) e2 = pm_pick(s, E);
            int e3 = pm_pick(s, E);
            for (int g = 0; (e3 == e1 || e3 == e2) && g < kMaxRejections; ++g) e3 = pm_pick(s, E);
            const uint8_t t = m.sl[e1];
            touched = (1ull << t) | (1ull << m.sl[e2]) | (1ull << m.sl[e3]);
            m.sl[e1] = m.sl[e2];
            m.sl[e2] = m.sl[e3];
            m.sl[e3] = t;
        }
        rng[p] = s;
        m.flags[0] = (uint32_t)touched;
        m.flags[1] = (uint32_t)(touched >> 32);
    }
    __syncthreads();
    const uint64_t touched = (uint64_t)m.flags[0] | ((uint64_t)m.flags[1] << 32);
    build_buckets(pb, m, lane);
    assign_touched(pb, m, touched, lane);
    store_row(slot + p * E, m.sl, E, lane);
    store_row(room + p * E, m.rr, E, lane);
}

static int tile_stride(int E) { return (E + 3) & ~3; }

int launch_assign_masked(const tt_problem* p, const uint8_t* slot, uint8_t* room, int P, const uint8_t* mask,
                         uint8_t bit, hipStream_t st) {
    const int nw = match_wide(p->R) ? kWideWaves : 1;
    const size_t lds = match_scratch_bytes(p->E, p->R, nw);
    if (lds > 160 * 1024) { set_error("instance too large for the matcher"); return TT_ERR_LIMIT; }
    const int threads = 64 * nw;
    hipLaunchKernelGGL(assign_rooms_kernel, dim3(P), dim3(threads), lds, st, p->dev, slot, room, P, mask, bit);
    return check_hip(hipGetLastError(), "assign_rooms launch");
}

int launch_mutation_masked(const tt_problem* p, uint8_t* slot, uint8_t* room, int64_t* rng, int P,
                           const uint8_t* mask, uint8_t bit, hipStream_t st) {
    const size_t lds = match_scratch_bytes(p->E, p->R);
    if (lds > 160 * 1024) { set_error("instance too large for the matcher"); return TT_ERR_LIMIT; }
    hipLaunchKernelGGL(mutation_kernel, dim3(P), dim3(64), lds, st, p->dev, slot, room, rng, P, mask, bit);
    return check_hip(hipGetLastError(), "mutation launch");
}

static int launch_assign(const tt_problem* p, const uint8_t* slot, uint8_t* room, int P, hipStream_t st) {
    return launch_assign_masked(p, slot, room, P, nullptr, 0, st);
}

}  // namespace ttga

using namespace ttga;

extern "C" int tt_assign_rooms(const tt_problem* p, const uint8_t* slot, uint8_t* room, int P, void* stream) {
    int rc = check_pop_args(p, P, slot, room);
    if (rc || P == 0) return rc;
    if ((rc = use_device(p))) return rc;
    return launch_assign(p, slot, room, P, (hipStream_t)stream);
}

extern "C" int tt_random_init(const tt_problem* p, int64_t* rng, uint8_t* slot, uint8_t* room, int P, void* stream) {
    int rc = check_pop_args(p, P, slot, room);
    if (rc || P == 0) return rc;
    if (!rng) { set_error("null rng buffer"); return TT_ERR_INVALID; }
    if ((rc = use_device(p))) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int SP = tile_stride(p->E);
    if ((size_t)64 * SP > 160 * 1024) { set_error("instance too large"); return TT_ERR_LIMIT; }
    hipLaunchKernelGGL(rand_slots_kernel, dim3((P + 63) / 64), dim3(64), (size_t)64 * SP, st, p->E, rng, slot, P, SP);
    if ((rc = check_hip(hipGetLastError(), "rand_slots launch"))) return rc;
    return launch_assign(p, slot, room, P, st);
}

extern "C" int tt_crossover(const tt_problem* p, const uint8_t* slot1, const uint8_t* slot2, int64_t* rng,
                            uint8_t* slot, uint8_t* room, int P, void* stream) {
    int rc = check_pop_args(p, P, slot1, slot2);
    if (rc || P == 0) return rc;
    if (!rng || !slot || !room) { set_error("null buffer"); return TT_ERR_INVALID; }
    if ((rc = use_device(p))) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int SP = tile_stride(p->E);
    if ((size_t)128 * SP > 160 * 1024) { set_error("instance too large"); return TT_ERR_LIMIT; }
    hipLaunchKernelGGL(crossover_slots_kernel, dim3((P + 63) / 64), dim3(64), (size_t)128 * SP, st, p->E, slot1,
                       slot2, rng, slot, P, SP);
    if ((rc = check_hip(hipGetLastError(), "crossover launch"))) return rc;
    return launch_assign(p, slot, room, P, st);
}

extern "C" int tt_mutation(const tt_problem* p, uint8_t* slot, uint8_t* room, int64_t* rng, int P, void* stream) {
    int rc = check_pop_args(p, P, slot, room);
    if (rc || P == 0) return rc;
    if (!rng) { set_error("null rng buffer"); return TT_ERR_INVALID; }
    if ((rc = use_device(p))) return rc;
    return launch_mutation_masked(p, slot, room, rng, P, nullptr, 0, (hipStream_t)stream);
}

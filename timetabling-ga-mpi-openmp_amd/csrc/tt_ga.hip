// GA generation primitives, batched over the children of one generation
// (ga.cpp:543-585 per child; C children are bred from the same population
// snapshot, the batched counterpart of the reference's OpenMP threads):
//
//   tt_ga_breed    per child c, on its own stream rng[c] (A.6 order):
//                    [3*E draws of the three discarded RandomInitialSolution, ga.cpp:543-548]
//                    parent a = selection5(pop), parent b = selection5(pop)   (ga.cpp:129-145,551-552)
//                    next() < p_cross ? crossover(a, b) : copy of a         (ga.cpp:562-566)
//                    next() < p_mut   ? randomMove                           (ga.cpp:569-571)
//   tt_ga_replace  children overwrite positions N-C..N-1 (ga.cpp:582 with
//                  C = 1), then the population is sorted by penalty
//                  ascending (ga.cpp:583); ties keep position order.
#include <algorithm>

#include "tt_internal.h"
#include "tt_match.h"

namespace ttga {

constexpr uint8_t kFlagCross = 1, kFlagMutate = 2;

// ---------------------------------------------------------------- breed
// One wave per child. Every lane replays the child's short sequential draws
// (the 3E discarded draws as one Park-Miller jump, the ten selection5 picks,
// the crossover and mutation draws); the E crossover picks, one per event,
// are drawn 64 at a time: event e = 64b + l takes state * 16807^(e+1), i.e.
// lane l multiplies its 16807^(l+1) by 16807^(64b) -- the same states the
// sequential loop would produce (Random.cc:27-37 for in-range states). The
// wave then writes its child row with coalesced byte stores.
__global__ __launch_bounds__(256) void breed_kernel(int E, const uint8_t* __restrict__ pop_slot,
                                                    const uint8_t* __restrict__ pop_room,
                                                    const int32_t* __restrict__ pen, int N,
                                                    int64_t* __restrict__ rng, int C, double p_cross, double p_mut,
                                                    int skip_init, uint32_t jump_skip, uint32_t jump_e,
                                                    uint8_t* __restrict__ child_slot, uint8_t* __restrict__ child_room,
                                                    uint8_t* __restrict__ flags) {
    const int lane = threadIdx.x & 63;
    const long ch = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ch >= C) return;                              // wave-uniform
    int64_t s = rng[ch];
    if (skip_init) {
        // the 3E discarded draws (ga.cpp:543-548): the first by Schrage (it brings an
        // out-of-range seed into range), the other 3E-1 as one jump
        pm_next(s);
        if ((uint64_t)s < kPmM)
            s = pm_mulmod((uint32_t)s, jump_skip);
        else
            for (int k = 1; k < 3 * E; ++k) pm_next(s);
    }
    int best[2];
    for (int q = 0; q < 2; ++q) {                     // selection5 (ga.cpp:129-145)
        int b = pm_pick(s, N);
        for (int i = 1; i < 5; ++i) {
            const int t = pm_pick(s, N);
            if ((uint32_t)pen[t] < (uint32_t)pen[b]) b = t;   // an invalid genome (-1) never wins
        }
        best[q] = b;
    }
    const uint8_t* sa = pop_slot + (long)best[0] * E;
    const uint8_t* sb = pop_slot + (long)best[1] * E;
    uint8_t* cs = child_slot + ch * E;
    uint8_t f = 0;
    if (pm_next(s) < p_cross) {                       // crossover (Solution.cpp:896-903)
        f |= kFlagCross;
        const uint32_t base = (uint32_t)s;            // in range: ten draws were taken
        const uint32_t a64 = pm_pow(64);
        uint32_t cur = pm_mulmod(base, pm_pow(lane + 1));
        for (int e = lane; e - lane < E; e += 64) {   // wave-uniform trip count
            const bool take_a = __dmul_rn(1.0 / 2147483647.0, (double)cur) < 0.5;
            if (e < E) cs[e] = take_a ? sa[e] : sb[e];
            cur = pm_mulmod(cur, a64);
        }
        s = pm_mulmod(base, jump_e);                  // the state after the E picks
    } else {
        const uint8_t* ra = pop_room + (long)best[0] * E;
        uint8_t* cr = child_room + ch * E;
        for (int e = lane; e < E; e += 64) { cs[e] = sa[e]; cr[e] = ra[e]; }
    }
    if (pm_next(s) < p_mut) f |= kFlagMutate;
    if (lane == 0) {
        rng[ch] = s;
        flags[ch] = f;
    }
}

// 16807^n mod (2^31 - 1) on the host (the breed jumps)
static uint32_t host_pm_pow(long n) {
    uint64_t r = 1, b = 16807;
    for (; n > 0; n >>= 1) {
        if (n & 1) r = r * b % 2147483647ull;
        b = b * b % 2147483647ull;
    }
    return (uint32_t)r;
}

// ---------------------------------------------------------------- replace + sort
// (penalty, position) as one u64; penalties compare as unsigned, so the -1 of an
// invalid genome (tt_eval's sentinel; valid penalties are >= 0) sorts last
__device__ __forceinline__ uint64_t sort_key(int32_t penalty, int pos) {
    return ((uint64_t)(uint32_t)penalty << 32) | (uint32_t)pos;
}

// keys of the merged population: positions < N-C from pop, the rest from the children
__global__ void replace_keys_kernel(const int32_t* __restrict__ pen, const int32_t* __restrict__ cpen, int N, int C,
                                    int NP, uint64_t* __restrict__ keys) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= NP) return;
    if (i >= N) { keys[i] = ~0ull; return; }
    const int k = N - C;
    keys[i] = sort_key(i < k ? pen[i] : cpen[i - k], i);
}

// bitonic sort of NP (power of two) u64 keys: one workgroup in LDS when NP <= 4096 ...
__global__ __launch_bounds__(1024) void bitonic_lds_kernel(uint64_t* __restrict__ keys, int NP) {
    __shared__ uint64_t sk[4096];
    for (int i = threadIdx.x; i < NP; i += blockDim.x) sk[i] = keys[i];
    __syncthreads();
    for (int k = 2; k <= NP; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < NP; i += blockDim.x) {
                const int l = i ^ j;
                if (l > i) {
                    const uint64_t x = sk[i], y = sk[l];
                    const bool up = (i & k) == 0;
                    if ((x > y) == up) { sk[i] = y; sk[l] = x; }
                }
            }
            __syncthreads();
        }
    }
    for (int i = threadIdx.x; i < NP; i += blockDim.x) keys[i] = sk[i];
}

// ... above that, tiles of kSortTile keys in LDS: bitonic_tile_kernel runs, per
// tile, the stages k <= kSortTile completely (full) or, for a stage k above the
// tile, its steps j < kSortTile (after the global steps j >= kSortTile). The
// direction of a pair is (i & k) of its global index i, as in one global pass.
constexpr int kSortTile = 8192;
__global__ __launch_bounds__(1024) void bitonic_tile_kernel(uint64_t* __restrict__ keys, int k_stage) {
    __shared__ uint64_t sk[kSortTile];
    const long base = (long)blockIdx.x * kSortTile;
    for (int i = threadIdx.x; i < kSortTile; i += 1024) sk[i] = keys[base + i];
    __syncthreads();
    auto step = [&](int k, int j) {
        for (int q = threadIdx.x; q < kSortTile / 2; q += 1024) {
            const int i = ((q & ~(j - 1)) << 1) | (q & (j - 1)), l = i + j;
            const uint64_t x = sk[i], y = sk[l];
            const bool up = ((base + i) & k) == 0;
            if ((x > y) == up) { sk[i] = y; sk[l] = x; }
        }
        __syncthreads();
    };
    if (k_stage == 0) {
        for (int k = 2; k <= kSortTile; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) step(k, j);
    } else {
        for (int j = kSortTile >> 1; j > 0; j >>= 1) step(k_stage, j);
    }
    for (int i = threadIdx.x; i < kSortTile; i += 1024) keys[base + i] = sk[i];
}

// one global pass of a (k, j) step with j >= kSortTile
__global__ void bitonic_step_kernel(uint64_t* __restrict__ keys, int NP, int k, int j) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= NP) return;
    const int l = i ^ j;
    if (l > i) {
        const uint64_t x = keys[i], y = keys[l];
        const bool up = (i & k) == 0;
        if ((x > y) == up) { keys[i] = y; keys[l] = x; }
    }
}

// ---- merge form of the sort (TT_GA_MERGE): the survivors (positions < k = N-C)
// of a population that a previous tt_ga_replace left sorted are already in key
// order, so the sorted merged population is the merge of them with the C
// children's keys sorted on their own (one workgroup in LDS for C <= kSortTile).
// Keys are unique (positions), so the merge equals the full sort. The survivors'
// order is checked on the device; when it does not hold (a migrant written into
// pop[N-2] survives when C = 1) a one-workgroup full sort runs instead. C = 0
// (the initial sort) takes the tiled sort directly.
#ifndef TT_GA_MERGE
#define TT_GA_MERGE 1
#endif

// kPrepBlocks workgroups: flag[g] = 1 when workgroup g's share of the survivors
// is in key order (all of them together: the survivors are); ckeys = the
// children's keys (padded to CP), sorted by the next launch
constexpr int kPrepBlocks = 64;
__global__ __launch_bounds__(256) void replace_prep_kernel(const int32_t* __restrict__ pen,
                                                           const int32_t* __restrict__ cpen, int N, int C, int CP,
                                                           uint64_t* __restrict__ ckeys, int32_t* __restrict__ flag) {
    const int k = N - C;
    const int gt = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
    for (int i = gt; i < CP; i += nth) ckeys[i] = i < C ? sort_key(cpen[i], k + i) : ~0ull;
    bool ok = true;
    for (int i = gt; i + 1 < k; i += nth) ok &= (uint32_t)pen[i] <= (uint32_t)pen[i + 1];
    ok = __syncthreads_and(ok);
    if (threadIdx.x == 0) flag[blockIdx.x] = ok ? 1 : 0;
}
// every workgroup's flag set (call with blockDim >= kPrepBlocks, every thread)
__device__ __forceinline__ bool survivors_sorted(const int32_t* flag) {
    return __syncthreads_and(threadIdx.x < kPrepBlocks ? flag[threadIdx.x] != 0 : true);
}

// merge path: output i takes the i-th smallest of survivors (pen[a], a) and ckeys
__global__ void replace_merge_kernel(const int32_t* __restrict__ pen, int N, int C, const uint64_t* __restrict__ ckeys,
                                     const int32_t* __restrict__ flag, uint64_t* __restrict__ mkeys) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (!survivors_sorted(flag) || i >= N) return;
    const int k = N - C;
    int lo = max(0, i - C), hi = min(i, k);
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sort_key(pen[mid], mid) < ckeys[i - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    const int a = lo, b = i - a;
    const uint64_t ka = a < k ? sort_key(pen[a], a) : ~0ull, kb = b < C ? ckeys[b] : ~0ull;
    mkeys[i] = ka < kb ? ka : kb;
}

// the fallback: full bitonic sort of keys[0..NP) by one workgroup in global memory
// (keys, 8 B each, stay L2-resident); nothing to do when the merge ran
__global__ __launch_bounds__(1024) void replace_fallback_sort_kernel(const int32_t* __restrict__ pen,
                                                                     const int32_t* __restrict__ cpen, int C,
                                                                     uint64_t* __restrict__ keys, int NP,
                                                                     const int32_t* __restrict__ flag,
                                                                     uint64_t* __restrict__ mkeys, int N) {
    if (survivors_sorted(flag)) return;
    for (int i = threadIdx.x; i < NP; i += blockDim.x)          // the keys (replace_keys_kernel's)
        keys[i] = i >= N ? ~0ull : sort_key(i < N - C ? pen[i] : cpen[i - (N - C)], i);
    __threadfence_block();
    __syncthreads();
    for (int k = 2; k <= NP; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int q = threadIdx.x; q < NP / 2; q += blockDim.x) {
                const int i = ((q & ~(j - 1)) << 1) | (q & (j - 1)), l = i + j;
                const uint64_t x = keys[i], y = keys[l];
                if ((x > y) == ((i & k) == 0)) { keys[i] = y; keys[l] = x; }
            }
            __threadfence_block();
            __syncthreads();
        }
    for (int i = threadIdx.x; i < N; i += blockDim.x) mkeys[i] = keys[i];
}

// ascending sort of tiles of T u64 keys (T a power of two, 2*KPT <= T <= kSortTile),
// one workgroup of T/KPT threads per tile (tile blockIdx.x), the keys in registers
// (TT_SORT_REG): thread t holds keys KPT*t..KPT*t+KPT-1; bitonic steps with j < KPT
// run inside a thread, KPT <= j < 64*KPT between lanes of a wave (shuffles), larger
// j between waves through LDS (double-buffered: one barrier per step).
#ifndef TT_SORT_REG
#define TT_SORT_REG 1
#endif
template <int KPT>
__global__ __launch_bounds__(1024) void sort_reg_kernel(uint64_t* __restrict__ keys, int T) {
    __shared__ uint64_t buf[KPT == 8 ? 2 : 1][KPT == 8 ? kSortTile : 1];
    keys += (size_t)blockIdx.x * T;
    const int t = threadIdx.x, nt = T / KPT;
    const bool own = t < nt;
    uint64_t v[KPT];
#pragma unroll
    for (int a = 0; a < KPT; ++a) v[a] = own ? keys[KPT * t + a] : ~0ull;
    int par = 0;
    for (int k = 2; k <= T; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {                 // uniform
            if (j >= KPT) {
                const int tj = j / KPT;                        // partner thread t ^ tj
                uint64_t w[KPT];
                if (KPT == 8 && tj >= 64) {                    // another wave: through LDS
                    if (own) {
#pragma unroll
                        for (int a = 0; a < KPT; ++a) buf[par][KPT * t + a] = v[a];
                    }
                    __syncthreads();
                    const int pt = own ? (t ^ tj) : t;
#pragma unroll
                    for (int a = 0; a < KPT; ++a) w[a] = buf[par][KPT * pt + a];
                    par ^= 1;
                } else {
#pragma unroll
                    for (int a = 0; a < KPT; ++a) w[a] = __shfl_xor(v[a], tj, 64);
                }
                const bool take_min = ((t & tj) == 0) == (((KPT * t) & k) == 0);
#pragma unroll
                for (int a = 0; a < KPT; ++a) v[a] = take_min ? (v[a] < w[a] ? v[a] : w[a]) : (v[a] < w[a] ? w[a] : v[a]);
            } else {
                // in-thread compare-exchanges with constant register indices (a runtime
                // index would put v[] in indexed-register mode); branch-free selects
                auto cx = [&](uint64_t& x, uint64_t& y, int a) {
                    const bool u = ((KPT * t + a) & k) == 0;
                    const uint64_t lo = x < y ? x : y, hi = x < y ? y : x;
                    x = u ? lo : hi;
                    y = u ? hi : lo;
                };
                if constexpr (KPT == 8) {
                    if (j == 4) {
                        cx(v[0], v[4], 0); cx(v[1], v[5], 1); cx(v[2], v[6], 2); cx(v[3], v[7], 3);
                    } else if (j == 2) {
                        cx(v[0], v[2], 0); cx(v[1], v[3], 1); cx(v[4], v[6], 4); cx(v[5], v[7], 5);
                    } else {
                        cx(v[0], v[1], 0); cx(v[2], v[3], 2); cx(v[4], v[5], 4); cx(v[6], v[7], 6);
                    }
                } else {
                    if (j == 2) {
                        cx(v[0], v[2], 0); cx(v[1], v[3], 1);
                    } else {
                        cx(v[0], v[1], 0); cx(v[2], v[3], 2);
                    }
                }
            }
        }
    }
    if (own) {
#pragma unroll
        for (int a = 0; a < KPT; ++a) keys[KPT * t + a] = v[a];
    }
}

// ---- tiled form of the sort (TT_SORT_RANK) for kRankTile*2 <= NP <= kSortTile:
// NP/kRankTile tiles sorted by one wave each (sort_reg_kernel<4>), then every key's
// rank in the whole array counted directly from the sorted tiles -- key x at
// position p of tile a has rank p + sum over tiles b < a of #{y <= x} + sum over
// tiles b > a of #{y < x} (stable, so padding duplicates get distinct ranks) --
// one lane per (key, tile), a binary search each, summed over the key's lanes.
// Two launches spread over NP/kRankTile and NP*NT/256 workgroups instead of one
// workgroup doing all 91 bitonic steps (64 us at 8,192 keys on one CU).
#ifndef TT_SORT_RANK
#define TT_SORT_RANK 1
#endif
constexpr int kRankTile = 256;

// rank of keys[i] among keys[0..NP) (tiles of kRankTile sorted); every thread of
// the group of NT lanes (NT = NP / kRankTile, a power of two <= 64) of key i calls it
__device__ __forceinline__ int tile_rank(const uint64_t* __restrict__ keys, int i, int NT, int b, uint64_t& x) {
    x = keys[i];
    const int a = i / kRankTile;
    int c;
    if (b == a) {
        c = i - a * kRankTile;
    } else {
        const uint64_t* tl = keys + (size_t)b * kRankTile;
        const bool le = b < a;                                 // earlier tiles: count y <= x
        c = 0;
#pragma unroll
        for (int s = kRankTile / 2; s >= 1; s >>= 1) {
            const uint64_t y = tl[c + s - 1];
            if (le ? y <= x : y < x) c += s;
        }
        const uint64_t y = tl[c];
        if (c < kRankTile && (le ? y <= x : y < x)) ++c;
    }
    for (int o = 1; o < NT; o <<= 1) c += __shfl_xor(c, o, 64);
    return c;
}

// sorted copy: out[rank(i)] = keys[i]
__global__ __launch_bounds__(256) void rank_scatter_kernel(const uint64_t* __restrict__ keys, int NP, int NT,
                                                           uint64_t* __restrict__ out) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = g / NT, b = g & (NT - 1);
    if (i >= NP) return;                                       // whole groups (NP*NT is a multiple of 256)
    uint64_t x;
    const int r = tile_rank(keys, i, NT, b, x);
    if (b == 0) out[r] = x;
}

// copy two rows of E bytes (slot and room), 512 bytes per lane block with all
// loads in flight before the stores
__device__ __forceinline__ void copy_rows2(uint8_t* __restrict__ d0, const uint8_t* __restrict__ s0,
                                           uint8_t* __restrict__ d1, const uint8_t* __restrict__ s1, int E,
                                           int lane) {
    for (int e0 = 0; e0 < E; e0 += 512) {
        uint8_t a[8], b[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int e = e0 + 64 * k + lane;
            a[k] = e < E ? s0[e] : 0;
            b[k] = e < E ? s1[e] : 0;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int e = e0 + 64 * k + lane;
            if (e < E) { d0[e] = a[k]; d1[e] = b[k]; }
        }
    }
}

// gather the sorted population into the work rows (one wave per row)
__global__ __launch_bounds__(64) void replace_gather_kernel(int E, int N, int C, const uint64_t* __restrict__ keys,
                                                            const uint8_t* __restrict__ ps, const uint8_t* __restrict__ pr,
                                                            const int32_t* __restrict__ ph, const int32_t* __restrict__ psc,
                                                            const uint8_t* __restrict__ pf, const int32_t* __restrict__ pp,
                                                            const uint8_t* __restrict__ cs, const uint8_t* __restrict__ cr,
                                                            const int32_t* __restrict__ ch, const int32_t* __restrict__ csc,
                                                            const uint8_t* __restrict__ cf, const int32_t* __restrict__ cp,
                                                            uint8_t* __restrict__ ws, uint8_t* __restrict__ wr,
                                                            int32_t* __restrict__ wm, int32_t* __restrict__ best_src) {
    const int i = blockIdx.x;
    const int src = (int)(keys[i] & 0xFFFFFFFFu);
    if (i == 0 && threadIdx.x == 0) *best_src = src;          // the new pop[0]'s merged position
    const int k = N - C;
    const bool child = src >= k;
    const int r = child ? src - k : src;
    const uint8_t* s = (child ? cs : ps) + (long)r * E;
    const uint8_t* m = (child ? cr : pr) + (long)r * E;
    copy_rows2(ws + (long)i * E, s, wr + (long)i * E, m, E, threadIdx.x);
    if (threadIdx.x == 0) {
        wm[4 * i + 0] = child ? ch[r] : ph[r];
        wm[4 * i + 1] = child ? csc[r] : psc[r];
        wm[4 * i + 2] = child ? cf[r] : pf[r];
        wm[4 * i + 3] = child ? cp[r] : pp[r];
    }
}

__global__ __launch_bounds__(64) void replace_scatter_kernel(int E, const uint8_t* __restrict__ ws,
                                                             const uint8_t* __restrict__ wr,
                                                             const int32_t* __restrict__ wm, uint8_t* __restrict__ ps,
                                                             uint8_t* __restrict__ pr, int32_t* __restrict__ ph,
                                                             int32_t* __restrict__ psc, uint8_t* __restrict__ pf,
                                                             int32_t* __restrict__ pp) {
    const int i = blockIdx.x;
    copy_rows2(ps + (long)i * E, ws + (long)i * E, pr + (long)i * E, wr + (long)i * E, E, threadIdx.x);
    if (threadIdx.x == 0) {
        ph[i] = wm[4 * i + 0];
        psc[i] = wm[4 * i + 1];
        pf[i] = (uint8_t)wm[4 * i + 2];
        pp[i] = wm[4 * i + 3];
    }
}

// keys for a longest-expected-first order: larger key first, ties by index,
// negative keys (invalid genomes) last; padding keys sort after all
__global__ void lpt_keys_kernel(const int32_t* __restrict__ key, int n, int NP, uint64_t* __restrict__ keys) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= NP) return;
    if (i >= n) { keys[i] = ~0ull; return; }
    const int32_t k = key[i];
    const uint32_t hi = k < 0 ? 0xFFFFFFFEu : (uint32_t)(0x7FFFFFFF - k);
    keys[i] = ((uint64_t)hi << 32) | (uint32_t)i;
}

__global__ void lpt_order_kernel(const uint64_t* __restrict__ keys, int n, int32_t* __restrict__ order) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) order[i] = (int32_t)(uint32_t)keys[i];
}

// order from tile-sorted keys: order[rank(i)] = index of key i (padding ranks >= n)
__global__ __launch_bounds__(256) void lpt_rank_order_kernel(const uint64_t* __restrict__ keys, int NP, int NT, int n,
                                                             int32_t* __restrict__ order) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = g / NT, b = g & (NT - 1);
    if (i >= NP) return;
    uint64_t x;
    const int r = tile_rank(keys, i, NT, b, x);
    if (b == 0 && r < n) order[r] = (int32_t)(uint32_t)x;
}

static int pow2_at_least(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace ttga

using namespace ttga;

// ascending bitonic sort of NP (a power of two) u64 keys on stream st
static void sort_keys(uint64_t* keys, int NP, hipStream_t st) {
    if (TT_SORT_REG && NP >= 8 && NP <= kSortTile) {
        hipLaunchKernelGGL(sort_reg_kernel<8>, dim3(1), dim3(std::max(64, NP / 8)), 0, st, keys, NP);
        return;
    }
    if (NP <= 4096) {
        hipLaunchKernelGGL(bitonic_lds_kernel, dim3(1), dim3(std::min(NP, 1024)), 0, st, keys, NP);
        return;
    }
    // NP / kSortTile tiles: 1 + sum over the stages above the tile of (global steps + 1)
    // launches (10 at NP = 65,536) instead of one per (k, j) step (136)
    const int tiles = NP / kSortTile;
    hipLaunchKernelGGL(bitonic_tile_kernel, dim3(tiles), dim3(1024), 0, st, keys, 0);
    for (int k = 2 * kSortTile; k <= NP; k <<= 1) {
        for (int j = k >> 1; j >= kSortTile; j >>= 1)
            hipLaunchKernelGGL(bitonic_step_kernel, dim3((NP + 255) / 256), dim3(256), 0, st, keys, NP, k, j);
        hipLaunchKernelGGL(bitonic_tile_kernel, dim3(tiles), dim3(1024), 0, st, keys, k);
    }
}

// launched from tt_rooms.hip (masked variants of the matcher and of mutation)
namespace ttga {
int launch_assign_masked(const tt_problem* p, const uint8_t* slot, uint8_t* room, int P, const uint8_t* mask,
                         uint8_t bit, hipStream_t st);
int launch_mutation_masked(const tt_problem* p, uint8_t* slot, uint8_t* room, int64_t* rng, int P,
                           const uint8_t* mask, uint8_t bit, hipStream_t st);
}  // namespace ttga

extern "C" int tt_ga_breed(const tt_problem* p, const uint8_t* pop_slot, const uint8_t* pop_room,
                           const int32_t* pop_penalty, int N, int64_t* rng, int C, double p_cross, double p_mut,
                           int skip_init_draws, uint8_t* child_slot, uint8_t* child_room, uint8_t* child_flags,
                           void* stream) {
    int rc = check_pop_args(p, C, child_slot, child_room);
    if (rc) return rc;
    if (N < 1 || !pop_slot || !pop_room || !pop_penalty || (C > 0 && (!rng || !child_flags))) {
        set_error("tt_ga_breed: bad population arguments");
        return TT_ERR_INVALID;
    }
    if (C == 0) return TT_OK;
    if ((rc = use_device(p))) return rc;
    hipStream_t st = (hipStream_t)stream;
    const uint32_t jump_skip = host_pm_pow(3L * p->E - 1), jump_e = host_pm_pow(p->E);
    hipLaunchKernelGGL(breed_kernel, dim3((C + 3) / 4), dim3(256), 0, st, p->E, pop_slot, pop_room, pop_penalty, N,
                       rng, C, p_cross, p_mut, skip_init_draws, jump_skip, jump_e, child_slot, child_room, child_flags);
    if ((rc = check_hip(hipGetLastError(), "breed launch"))) return rc;
    if ((rc = launch_assign_masked(p, child_slot, child_room, C, child_flags, kFlagCross, st))) return rc;
    return launch_mutation_masked(p, child_slot, child_room, rng, C, child_flags, kFlagMutate, st);
}

// NP keys in [2*kRankTile, kSortTile]: sorted by tiles + ranks (TT_SORT_RANK)
static bool use_rank_sort(int NP) { return TT_SORT_RANK && NP >= 2 * kRankTile && NP <= kSortTile; }
// the tiles of the rank sort (ranks are then counted by the caller's kernel)
static void sort_rank_tiles(uint64_t* keys, int NP, hipStream_t st) {
    hipLaunchKernelGGL(sort_reg_kernel<4>, dim3(NP / kRankTile), dim3(kRankTile / 4), 0, st, keys, kRankTile);
}

// work layout: sort keys [pow2(N)] u64 | slot rows [N][E] | room rows [N][E] |
// meta [N][4] i32 | the source slot (256 B, written only by tt_ga_replace) |
// merged keys [N] u64 | child keys [kSortTile] u64 | merge flag (256 B) |
// sorted child keys [kSortTile] u64
static size_t work_source_offset(int N, int E) {
    const size_t NP = (size_t)pow2_at_least(N);
    return align256(8 * NP) + 2 * align256((size_t)N * E) + align256(16 * (size_t)N);
}
static size_t work_merge_offset(int N, int E) { return work_source_offset(N, E) + 256; }

extern "C" size_t tt_ga_work_bytes(int N, int E) {
    if (N < 1 || E < 1) return 0;
    return work_merge_offset(N, E) + align256(8 * (size_t)N) + 16 * (size_t)kSortTile + 256;
}

extern "C" size_t tt_ga_work_source_offset(int N, int E) {
    if (N < 1 || E < 1) return 0;
    return work_source_offset(N, E);
}

extern "C" int tt_ga_replace(const tt_problem* p, uint8_t* pop_slot, uint8_t* pop_room, int32_t* pop_hcv,
                             int32_t* pop_scv, uint8_t* pop_feasible, int32_t* pop_penalty, int N,
                             const uint8_t* child_slot, const uint8_t* child_room, const int32_t* child_hcv,
                             const int32_t* child_scv, const uint8_t* child_feasible, const int32_t* child_penalty,
                             int C, void* work, void* stream) {
    if (!p || N < 1 || C < 0 || C > N || !work || !pop_slot || !pop_room || !pop_hcv || !pop_scv || !pop_feasible ||
        !pop_penalty || (C > 0 && (!child_slot || !child_room || !child_hcv || !child_scv || !child_feasible ||
                                   !child_penalty))) {
        set_error("tt_ga_replace: bad arguments");
        return TT_ERR_INVALID;
    }
    int rc = use_device(p);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int E = p->E, NP = pow2_at_least(N);
    uint8_t* w = (uint8_t*)work;
    uint64_t* keys = (uint64_t*)w;
    uint8_t* ws = w + align256(8 * (size_t)NP);
    uint8_t* wr = ws + align256((size_t)N * E);
    int32_t* wm = (int32_t*)(wr + align256((size_t)N * E));
    const uint64_t* sorted = keys;
    // C = 0 sorts a population with no order to rely on (the initial sort,
    // ga.cpp:433-434): the multi-workgroup sort, not the merge path's
    // one-workgroup fallback (which a generation meets only when a migrant
    // survives out of order, C = 1)
    if (TT_GA_MERGE && C > 0 && C <= kSortTile) {
        uint64_t* mkeys = (uint64_t*)(w + work_merge_offset(N, E));
        uint64_t* ckeys = (uint64_t*)((uint8_t*)mkeys + align256(8 * (size_t)N));
        int32_t* flag = (int32_t*)(ckeys + kSortTile);
        const int CP = pow2_at_least(std::max(C, 2));
        hipLaunchKernelGGL(replace_prep_kernel, dim3(kPrepBlocks), dim3(256), 0, st, pop_penalty, child_penalty, N, C, CP,
                           ckeys, flag);
        const uint64_t* csorted = ckeys;
        if (use_rank_sort(CP)) {
            uint64_t* cs2 = (uint64_t*)((uint8_t*)flag + 256);
            const int NT = CP / kRankTile;
            sort_rank_tiles(ckeys, CP, st);
            hipLaunchKernelGGL(rank_scatter_kernel, dim3(CP * NT / 256), dim3(256), 0, st, ckeys, CP, NT, cs2);
            csorted = cs2;
        } else {
            sort_keys(ckeys, CP, st);
        }
        hipLaunchKernelGGL(replace_merge_kernel, dim3((N + 255) / 256), dim3(256), 0, st, pop_penalty, N, C, csorted,
                           flag, mkeys);
        hipLaunchKernelGGL(replace_fallback_sort_kernel, dim3(1), dim3(1024), 0, st, pop_penalty, child_penalty, C, keys,
                           NP, flag, mkeys, N);
        sorted = mkeys;
    } else {
        hipLaunchKernelGGL(replace_keys_kernel, dim3((NP + 255) / 256), dim3(256), 0, st, pop_penalty, child_penalty, N,
                           C, NP, keys);
        sort_keys(keys, NP, st);
    }
    hipLaunchKernelGGL(replace_gather_kernel, dim3(N), dim3(64), 0, st, E, N, C, sorted, pop_slot, pop_room, pop_hcv,
                       pop_scv, pop_feasible, pop_penalty, child_slot, child_room, child_hcv, child_scv, child_feasible,
                       child_penalty, ws, wr, wm, (int32_t*)(w + work_source_offset(N, E)));
    hipLaunchKernelGGL(replace_scatter_kernel, dim3(N), dim3(64), 0, st, E, ws, wr, wm, pop_slot, pop_room, pop_hcv,
                       pop_scv, pop_feasible, pop_penalty);
    return check_hip(hipGetLastError(), "tt_ga_replace launch");
}

extern "C" int tt_lpt_order(const tt_problem* p, const int32_t* key, int n, int32_t* order, void* work, void* stream) {
    if (!p || n < 0 || (n > 0 && (!key || !order || !work))) {
        set_error("tt_lpt_order: bad arguments");
        return TT_ERR_INVALID;
    }
    if (n == 0) return TT_OK;
    int rc = use_device(p);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int NP = pow2_at_least(n);
    uint64_t* keys = (uint64_t*)work;
    hipLaunchKernelGGL(lpt_keys_kernel, dim3((NP + 255) / 256), dim3(256), 0, st, key, n, NP, keys);
    if (use_rank_sort(NP)) {
        const int NT = NP / kRankTile;
        sort_rank_tiles(keys, NP, st);
        hipLaunchKernelGGL(lpt_rank_order_kernel, dim3(NP * NT / 256), dim3(256), 0, st, keys, NP, NT, n, order);
        return check_hip(hipGetLastError(), "tt_lpt_order launch");
    }
    sort_keys(keys, NP, st);
    hipLaunchKernelGGL(lpt_order_kernel, dim3((n + 255) / 256), dim3(256), 0, st, keys, n, order);
    return check_hip(hipGetLastError(), "tt_lpt_order launch");
}

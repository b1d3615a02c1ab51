// Wave-level room assignment: Solution::assignRooms (Solution.cpp:772-891).
//
// The reference builds, per timeslot, a flow network source(1) -> events
// (2..N+1) -> rooms (N+2..N+R+1) -> sink (V) with unit capacities and runs a
// priority-first search (networkFlow) until no augmenting path remains. With
// unit capacities every reachable node gets priority value -9 and unseen
// nodes -10, so the search always expands the LOWEST-INDEX fringe node: all
// fringe events (ascending), then fringe rooms (ascending), the sink last;
// a node's dad is the first visited node with a residual edge to it, and the
// augmenting path is fixed the moment the first FREE room is visited (its dad
// chain never changes afterwards). This file replays exactly that search on
// 64-bit bitsets (events of the slot, rooms), one LANE PER TIMESLOT, one WAVE
// PER INDIVIDUAL. Read-out (Solution.cpp:802-830): matched events take their
// room; unmatched events take the first possible room unless a possible room
// is free (busy[] starts at 0), and an event with no possible room
// keeps the carried-over lessBusy (initially 0, declared once per call).
#pragma once
#include "tt_common.h"

namespace ttga {

constexpr uint8_t kNone = 0xFF;

#ifndef TT_BUCKETS_CHUNK
#define TT_BUCKETS_CHUNK 1
#endif

// TT_ROOMS_WAVE: assign_touched matches a slot by the whole wave
// (wave_match_slot) instead of one slot per lane (match_slot / match_slot_reg:
// lane-serial searches that wait on LDS at every step), except the many small
// slots of a whole-row assignment on an instance of <= 16 rooms, which stay one
// per lane in registers; slots of more than 64 events stay lane-serial.
#ifndef TT_ROOMS_WAVE
#define TT_ROOMS_WAVE 1
#endif
constexpr int kWaveSlots = 8;    // touched slots up to which every slot goes to the wave matcher

// Per-wave LDS scratch for one individual. Two layouts:
//  * R <= 16 (or TT_ROOMS_WAVE=0): every slot's possible-room masks, matched
//    rooms, room owners and dads, for one slot per lane;
//  * R > 16 ("wide", TT_ROOMS_WAVE): the wave matcher keeps its state in
//    registers and reads the possible rooms from the problem (L2-resident), so
//    the scratch holds the row, its buckets and, per wave, one crowded slot's
//    state for the lane-serial fallback: 4E + 2.4 KB per wave instead of
//    14E + 90R (syn: 11 KB for one wave, 18.5 KB for four, instead of 30 KB);
//    in assign_rooms_kernel kWideWaves waves share an individual and take its
//    slots t with t % kWideWaves == wave (syn, 65,536 rows: one wave 23.7 ms,
//    two 20.0, three 19.4, four 18.8; profiles/r06_ae_ab_rooms_waves.jsonl).
struct MatchScratch {
    uint8_t* sl;        // [E]     slot of each event
    uint8_t* rr;        // [E]     room of each event (output row)
    uint16_t* bev;      // [E]     events bucketed by slot, ascending inside a slot
    uint8_t* mr;        // [E]     matched room per bucket position (kNone)   wide: [waves][256], one slot
    uint64_t* pl;       // [E]     possible-room mask per bucket position    wide: [waves][256], one slot
    uint8_t* rm;        // [45*R]  event (bucket-local index) matched to each room   wide: [waves][R]
    uint8_t* dr;        // [45*R]  dad (bucket-local event) of each room in the search   wide: [waves][R]
    int32_t* bstart;    // [46]    bucket offsets
    uint32_t* tmp;      // [64]
    uint32_t* flags;    // [4]
    uint64_t* cm;       // [64]    per-slot lane masks of one 64-event chunk (build_buckets)
    bool wide;
};

__host__ __device__ inline bool match_wide(int R) { return TT_ROOMS_WAVE && R > 16; }
#ifndef TT_WIDE_WAVES
#define TT_WIDE_WAVES 4
#endif
constexpr int kWideWaves = TT_WIDE_WAVES;    // waves per individual in assign_rooms_kernel, wide layout

// nw: waves sharing the individual (wide layout: one crowded slot's state each)
__host__ __device__ inline size_t match_scratch_bytes(int E, int R, int nw = 1) {
    const bool wide = match_wide(R);
    const size_t nb = wide ? (size_t)nw * kMaxSlotEvents : (size_t)E;   // bucket positions with state
    const size_t nr = wide ? (size_t)nw * R : (size_t)kSlots * R;
    size_t b = 0;
    b += (size_t)E;                          // sl
    b += (size_t)E;                          // rr
    b = (b + 1) & ~(size_t)1;
    b += 2 * (size_t)E;                      // bev
    b += nb;                                 // mr
    b = (b + 7) & ~(size_t)7;
    b += 8 * nb;                             // pl
    b += 2 * nr;                             // rm, dr
    b = (b + 3) & ~(size_t)3;
    b += 4 * 46 + 4 * 64 + 4 * 4;            // bstart, tmp, flags
    b = (b + 7) & ~(size_t)7;
    b += 8 * 64;                             // cm
    return (b + 15) & ~(size_t)15;
}

__device__ inline MatchScratch carve_match_scratch(uint8_t* base, int E, int R, int nw = 1) {
    MatchScratch m;
    m.wide = match_wide(R);
    const size_t nb = m.wide ? (size_t)nw * kMaxSlotEvents : (size_t)E;
    const size_t nr = m.wide ? (size_t)nw * R : (size_t)kSlots * R;
    size_t b = 0;
    m.sl = base + b; b += E;
    m.rr = base + b; b += E;
    b = (b + 1) & ~(size_t)1;
    m.bev = (uint16_t*)(base + b); b += 2 * (size_t)E;
    m.mr = base + b; b += nb;
    b = (b + 7) & ~(size_t)7;
    m.pl = (uint64_t*)(base + b); b += 8 * nb;
    m.rm = base + b; b += nr;
    m.dr = base + b; b += nr;
    b = (b + 3) & ~(size_t)3;
    m.bstart = (int32_t*)(base + b); b += 4 * 46;
    m.tmp = (uint32_t*)(base + b); b += 4 * 64;
    m.flags = (uint32_t*)(base + b); b += 4 * 4;
    b = (b + 7) & ~(size_t)7;
    m.cm = (uint64_t*)(base + b);
    return m;
}

__device__ __forceinline__ int wave_inclusive_scan(int v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

// Bucket the events by slot, ascending event index inside each bucket
// (the order of timeslot_events lists, which are always kept sorted).
// All 64 lanes of the wave call this; sl[] must be filled.
// act: this wave does the work (a workgroup of several waves: the first; the
// others only meet the barriers).
__device__ inline void build_buckets(const DevProblem& pb, MatchScratch& m, int lane, bool act = true) {
    const int E = pb.E;
    if (act) m.tmp[lane] = 0u;
    __syncthreads();
    if (act)
        for (int e = lane; e < E; e += 64) {
            const int s = m.sl[e];
            if (s < kSlots) atomicAdd(&m.tmp[s], 1u);
        }
    __syncthreads();
    const int c = lane < kSlots ? (int)m.tmp[lane] : 0;
    const int incl = wave_inclusive_scan(c, lane);
    const int start = incl - c;
    if (act && lane < kSlots) m.bstart[lane] = start;
    if (act && lane == kSlots - 1) m.bstart[kSlots] = incl;
#if TT_BUCKETS_CHUNK
    // stable fill, 64 events at a time: each event sets its lane bit in its slot's
    // chunk mask; its place is the slot's running count plus the lower lanes of the
    // mask (ascending event order inside a bucket, as the lane walk below)
    if (act) m.cm[lane] = 0ull;
    int cur = start;                                  // lane t < 45: slot t's next position
    __syncthreads();
    for (int c0 = 0; c0 < E; c0 += 64) {
        const int e = c0 + lane;
        const int s = act && e < E ? m.sl[e] : 0xFF;
        if (s < kSlots) atomicOr((unsigned long long*)&m.cm[s], 1ull << lane);
        const int base = __shfl(cur, s < kSlots ? s : 0, 64);       // every lane takes part
        __syncthreads();
        if (s < kSlots) m.bev[base + __popcll(m.cm[s] & ((1ull << lane) - 1ull))] = (uint16_t)e;
        __syncthreads();
        if (act && lane < kSlots) {
            cur += __popcll(m.cm[lane]);
            m.cm[lane] = 0ull;
        }
        __syncthreads();
    }
#else
    // stable fill: lane t walks the slot row (broadcast reads) and keeps its events
    int pos = start;
    int e = 0;
    const int me = lane < kSlots ? lane : 0x100;     // lanes >= 45 never match a byte
    for (; e + 4 <= E; e += 4) {
        uint32_t w = (uint32_t)m.sl[e] | ((uint32_t)m.sl[e + 1] << 8) | ((uint32_t)m.sl[e + 2] << 16) |
                     ((uint32_t)m.sl[e + 3] << 24);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if ((int)((w >> (8 * k)) & 0xFFu) == me) m.bev[pos++] = (uint16_t)(e + k);
    }
    for (; e < E; ++e)
        if (m.sl[e] == me) m.bev[pos++] = (uint16_t)e;
    static_assert(TT_BUCKETS_CHUNK, "the lane walk has no act flag");
#endif
    __syncthreads();
    if (m.wide || !act) return;                        // wide: the wave matcher reads pb.poss itself
    const int nb = m.bstart[kSlots];
    for (int b0 = 0; b0 < nb; b0 += 512) {            // eight gathers in flight per block
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int b = b0 + 64 * k + lane;
            v[k] = b < nb ? pb.poss[m.bev[b]] : 0ull;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int b = b0 + 64 * k + lane;
            if (b < nb) m.pl[b] = v[k];
        }
    }
    __syncthreads();
}

template <int NW>
__device__ __forceinline__ int pop_lowest(uint64_t (&f)[NW]) {
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        if (f[w]) {
            const int b = __builtin_ctzll(f[w]);
            f[w] &= f[w] - 1;
            return 64 * w + b;
        }
    }
    return -1;
}

// Max-cardinality matching + read-out for one slot (N events, N <= 64*NW).
template <int NW>
__device__ void match_slot(int R, const uint16_t* ev, const uint64_t* pl, int N, uint8_t* mr, uint8_t* rm,
                           uint8_t* dr, uint8_t* rr) {
    uint64_t unm[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const int lo = 64 * w;
        unm[w] = N >= lo + 64 ? ~0ull : (N > lo ? ((1ull << (N - lo)) - 1ull) : 0ull);
    }
    for (int i = 0; i < N; ++i) mr[i] = kNone;
    uint64_t rmatched = 0;
    for (;;) {
        // networkFlow (Solution.cpp:852-891): lowest-index-first search from the source
        uint64_t se[NW], fe[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) { se[w] = unm[w]; fe[w] = unm[w]; }
        uint64_t sr = 0, fr = 0;
        int sink = -1;
        for (;;) {
            const int i = pop_lowest<NW>(fe);
            if (i >= 0) {                              // expand event i: forward residual edges
                const uint64_t own = mr[i] != kNone ? (1ull << mr[i]) : 0ull;
                uint64_t nr = pl[i] & ~sr & ~own;
                sr |= nr;
                fr |= nr;
                while (nr) {
                    const int j = __builtin_ctzll(nr);
                    nr &= nr - 1;
                    dr[j] = (uint8_t)i;
                }
                continue;
            }
            if (fr) {                                  // expand room j
                const int j = __builtin_ctzll(fr);
                fr &= fr - 1;
                if (!((rmatched >> j) & 1ull)) { sink = j; break; }   // free room: path to the sink is fixed
                const int i2 = rm[j];                  // reverse edge to its matched event
                const uint64_t b = 1ull << (i2 & 63);
#pragma unroll
                for (int w = 0; w < NW; ++w)
                    if (w == (i2 >> 6) && !(se[w] & b)) { se[w] |= b; fe[w] |= b; }
                continue;
            }
            break;
        }
        if (sink < 0) break;
        // maxMatching augmentation (Solution.cpp:836-849)
        int j = sink;
        for (;;) {
            const int i = dr[j];
            const int prev = mr[i];
            mr[i] = (uint8_t)j;
            rm[j] = (uint8_t)i;
            rmatched |= 1ull << j;
            if (prev == kNone) {
#pragma unroll
                for (int w = 0; w < NW; ++w)
                    if (w == (i >> 6)) unm[w] &= ~(1ull << (i & 63));
                break;
            }
            j = prev;
        }
    }
    // read-out and unplaced events (Solution.cpp:802-830)
    int less_busy = 0;
    for (int i = 0; i < N; ++i) {
        int r = mr[i];
        if (r == kNone) {
            const uint64_t ps = pl[i];
            if (ps) {
                less_busy = __builtin_ctzll(ps);
                if ((rmatched >> less_busy) & 1ull) {
                    const uint64_t fr2 = ps & ~rmatched;
                    if (fr2) less_busy = __builtin_ctzll(fr2);
                }
            }
            r = less_busy;
        }
        rr[ev[i]] = (uint8_t)r;
    }
}

// match_slot for N <= 32 events and R <= 16 rooms (TT_MATCH_REG) with the
// matching itself in registers: the matched room of each event as 4-bit fields
// (mr0: events 0-15, mr1: 16-31; valid while the event's bit is clear in unm)
// and the event matched to each room as 8-bit fields (rm0: rooms 0-7, rm1:
// 8-15). The lane-serial search then waits on LDS only for an event's
// possible rooms (and writes its dads there, read back on the augmenting path):
// a room expansion and the path's matched-room lookups are register selects.
// Same search, same result as match_slot.
#ifndef TT_MATCH_REG
#define TT_MATCH_REG 1
#endif
__device__ __forceinline__ uint32_t nib_get(uint64_t w0, uint64_t w1, int i) {
    return (uint32_t)(((i < 16 ? w0 : w1) >> (4 * (i & 15))) & 15ull);
}
__device__ __forceinline__ void nib_set(uint64_t& w0, uint64_t& w1, int i, uint32_t v) {
    const int sh = 4 * (i & 15);
    const uint64_t clr = ~(15ull << sh), put = (uint64_t)v << sh;
    if (i < 16) w0 = (w0 & clr) | put;
    else w1 = (w1 & clr) | put;
}
__device__ __forceinline__ uint32_t byte_get(uint64_t w0, uint64_t w1, int j) {
    return (uint32_t)(((j < 8 ? w0 : w1) >> (8 * (j & 7))) & 255ull);
}
__device__ __forceinline__ void byte_set(uint64_t& w0, uint64_t& w1, int j, uint32_t v) {
    const int sh = 8 * (j & 7);
    const uint64_t clr = ~(255ull << sh), put = (uint64_t)v << sh;
    if (j < 8) w0 = (w0 & clr) | put;
    else w1 = (w1 & clr) | put;
}

__device__ void match_slot_reg(const uint16_t* ev, const uint64_t* pl, int N, uint8_t* dr, uint8_t* rr) {
    uint32_t unm = N >= 32 ? ~0u : ((1u << N) - 1u);
    uint64_t mr0 = 0, mr1 = 0, rm0 = 0, rm1 = 0;
    uint32_t rmatched = 0;
    for (;;) {
        // networkFlow (Solution.cpp:852-891): lowest-index-first search from the source
        uint32_t se = unm, fe = unm, sr = 0, fr = 0;
        int sink = -1;
        for (;;) {
            if (fe) {                                  // expand event i: forward residual edges
                const int i = __builtin_ctz(fe);
                fe &= fe - 1;
                const uint32_t own = ((unm >> i) & 1u) ? 0u : (1u << nib_get(mr0, mr1, i));
                uint32_t nr = (uint32_t)pl[i] & ~sr & ~own;
                sr |= nr;
                fr |= nr;
                while (nr) {
                    const int j = __builtin_ctz(nr);
                    nr &= nr - 1;
                    dr[j] = (uint8_t)i;
                }
                continue;
            }
            if (fr) {                                  // expand room j
                const int j = __builtin_ctz(fr);
                fr &= fr - 1;
                if (!((rmatched >> j) & 1u)) { sink = j; break; }   // free room: path to the sink is fixed
                const uint32_t b = 1u << byte_get(rm0, rm1, j);     // reverse edge to its matched event
                if (!(se & b)) { se |= b; fe |= b; }
                continue;
            }
            break;
        }
        if (sink < 0) break;
        // maxMatching augmentation (Solution.cpp:836-849)
        int j = sink;
        for (;;) {
            const int i = dr[j];
            const bool was = !((unm >> i) & 1u);
            const int prev = (int)nib_get(mr0, mr1, i);
            nib_set(mr0, mr1, i, (uint32_t)j);
            byte_set(rm0, rm1, j, (uint32_t)i);
            rmatched |= 1u << j;
            if (!was) {
                unm &= ~(1u << i);
                break;
            }
            j = prev;
        }
    }
    // read-out and unplaced events (Solution.cpp:802-830)
    int less_busy = 0;
    for (int i = 0; i < N; ++i) {
        int r;
        if (!((unm >> i) & 1u)) {
            r = (int)nib_get(mr0, mr1, i);
        } else {
            const uint64_t ps = pl[i];
            if (ps) {
                less_busy = __builtin_ctzll(ps);
                if ((rmatched >> less_busy) & 1u) {
                    const uint64_t fr2 = ps & ~(uint64_t)rmatched;
                    if (fr2) less_busy = __builtin_ctzll(fr2);
                }
            }
            r = less_busy;
        }
        rr[ev[i]] = (uint8_t)r;
    }
}

// lane j of (lo, hi) = the 64-bit wave-uniform v. The lane select goes
// through M0 (gfx9 reads one SGPR per VALU instruction besides M0); the s_nop
// pads the M0 write (inline asm gets no hazard padding from the compiler).
// M0 is declared clobbered; no kernel that calls this uses LDS-DMA or movrel.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void writelane64(uint32_t& lo, uint32_t& hi, uint64_t v, int j) {
    asm volatile("s_mov_b32 m0, %4\n\ts_nop 1\n\tv_writelane_b32 %0, %2, m0\n\tv_writelane_b32 %1, %3, m0"
                 : "+v"(lo), "+v"(hi)
                 : "s"((uint32_t)v), "s"((uint32_t)(v >> 32)), "s"(j)
                 : "m0");
}
#pragma clang diagnostic pop

// One slot of N <= 64 events matched by the whole wave (the local search's
// match_task_wave without its bookkeeping): lane i holds event i's possible
// rooms pl (zero past N) and matched room mr; lane j holds room j's matched
// event rm, its possible rooms plr, its search dad dr, and the events that may
// use it (eor); the seen / fringe room sets are wave-uniform bitsets. Same
// search and read-out as match_slot (Solution.cpp:802-891):
//  * the search expands every fringe event before any room, so its first
//    stage (all unmatched events, ascending) is closed-form: the rooms seen are
//    those with an unmatched candidate, room j's dad its lowest one;
//  * the room stage pops fringe rooms ascending; a matched room's event is
//    expanded at once and can only discover unseen rooms, so every popped room
//    whose event discovers none is popped in bulk (one ballot), up to the
//    first that does or the lowest free room (the sink).
// Returns event lane's room (lanes < N).
__device__ __forceinline__ uint32_t wave_match_slot(int R, int N, uint64_t pl, int lane) {
    constexpr uint32_t NONE = 0xFFu;
    const uint32_t pl_lo = (uint32_t)pl, pl_hi = (uint32_t)(pl >> 32);
    uint32_t eor_lo = 0, eor_hi = 0;
    const int r1 = R < 32 ? R : 32;
    for (int j = 0; j < r1; ++j) writelane64(eor_lo, eor_hi, ballot((pl_lo >> j) & 1u), j);
    for (int j = 32; j < R; ++j) writelane64(eor_lo, eor_hi, ballot((pl_hi >> (j - 32)) & 1u), j);
    const uint64_t eor = ((uint64_t)eor_hi << 32) | eor_lo;
    uint32_t mr = NONE, rm = 0, dr = 0, plr_lo = 0, plr_hi = 0;
    uint64_t unm = N >= 64 ? ~0ull : ((1ull << N) - 1ull);
    uint64_t rmatched = 0;
    for (;;) {
        const uint64_t cand = eor & unm;                 // stage 1, closed form
        uint64_t sr = ballot(cand != 0ull), fr = sr;     // eor is zero on lanes >= R
        if (cand) dr = (uint32_t)__builtin_ctzll(cand);
        int sink = -1;
        for (;;) {                                       // stage 2, bulk pops
            const uint64_t freef = fr & ~rmatched;
            const uint64_t M = fr & (freef ? (freef & (0ull - freef)) - 1ull : ~0ull);
            const uint64_t plr = ((uint64_t)plr_hi << 32) | plr_lo;
            // M is uniform: one ballot over every room lane, then M's lanes kept
            const uint64_t disc = ballot((plr & ~sr) != 0ull) & M;
            if (!disc) {
                if (freef) sink = __builtin_ctzll(freef);
                break;
            }
            const int j = __builtin_ctzll(disc);
            fr &= ~(M & ((2ull << j) - 1ull));           // pops M's rooms up to j
            const int i2 = __builtin_amdgcn_readlane((int)rm, j);
            const uint64_t pli = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)plr_hi, j) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)plr_lo, j);
            const uint64_t nr = pli & ~sr;
            sr |= nr;
            fr |= nr;
            if ((nr >> lane) & 1ull) dr = (uint32_t)i2;
        }
        if (sink < 0) break;
        int j = sink;                                    // maxMatching augmentation (Solution.cpp:836-849)
        for (;;) {
            const int i = __builtin_amdgcn_readlane((int)dr, j);
            const uint32_t prev = (uint32_t)__builtin_amdgcn_readlane((int)mr, i);
            const uint32_t pi_lo = (uint32_t)__builtin_amdgcn_readlane((int)pl_lo, i);
            const uint32_t pi_hi = (uint32_t)__builtin_amdgcn_readlane((int)pl_hi, i);
            if (lane == i) mr = (uint32_t)j;
            if (lane == j) { rm = (uint32_t)i; plr_lo = pi_lo; plr_hi = pi_hi; }
            rmatched |= 1ull << j;
            if (prev == NONE) { unm &= ~(1ull << i); break; }
            j = (int)prev;
        }
    }
    // read-out (Solution.cpp:802-830): unplaced events, ascending, take the first
    // free possible room, else the first possible room; one with no possible room
    // keeps lessBusy carried over from the previous unplaced event (initially 0)
    const bool un = lane < N && mr == NONE;
    if (!ballot(un)) return mr;
    uint32_t v = 0;
    if (un && pl) {
        v = (uint32_t)__builtin_ctzll(pl);
        if ((rmatched >> v) & 1ull) {
            const uint64_t fr2 = pl & ~rmatched;
            if (fr2) v = (uint32_t)__builtin_ctzll(fr2);
        }
    }
    const uint64_t carriers = ballot(un && pl != 0ull);
    const uint64_t below = carriers & ((1ull << lane) - 1ull);
    const int src = below ? 63 - __builtin_clzll(below) : lane;
    const uint32_t carried = (uint32_t)__shfl((int)v, src, 64);
    return !un ? mr : (pl ? v : (below ? carried : 0u));
}

// Re-assign rooms for every slot t with bit t of `touched` set and a
// non-empty bucket. m.sl and m.rr hold the individual's row; rooms of
// untouched slots in m.rr are left as they are. Buckets must be built.
// wave w of nw: the slots t with t % nw == w (wide layout only).
__device__ inline void assign_touched(const DevProblem& pb, MatchScratch& m, uint64_t touched, int lane,
                                      int w = 0, int nw = 1) {
#if TT_ROOMS_WAVE
    const int R = pb.R;
    touched &= (1ull << kSlots) - 1ull;
    if (nw > 1) {                                       // this wave's slots: t % nw == w
        uint64_t wm = 0;
        for (int t = w; t < kSlots; t += nw) wm |= 1ull << t;
        touched &= wm;
    }
    if (!m.wide && __popcll(touched) > kWaveSlots) {
        // a whole row on a small instance: slots of <= 32 events one per lane, in
        // registers, all at once; the crowded ones go to the wave below
        bool mine = false;
        if (lane < kSlots && ((touched >> lane) & 1ull)) {
            const int b0 = m.bstart[lane];
            const int N = m.bstart[lane + 1] - b0;
            if (N <= 32) {
                mine = true;
                if (N > 0) match_slot_reg(m.bev + b0, m.pl + b0, N, m.dr + lane * R, m.rr);
            }
        }
        touched &= ~ballot(mine);
    }
    // the wave's slots one after another; the next slot's events and possible
    // rooms are loaded while the current one is matched
    int t = touched ? __builtin_ctzll(touched) : 0;
    int b0 = __builtin_amdgcn_readfirstlane(m.bstart[t]);
    int N = __builtin_amdgcn_readfirstlane(m.bstart[t + 1]) - b0;
    int ev = lane < N ? m.bev[b0 + lane] : 0;
    uint64_t pl = lane < N && N <= 64 ? (m.wide ? pb.poss[ev] : m.pl[b0 + lane]) : 0ull;
    while (touched) {
        touched &= touched - 1;
        const int tc = t, bc = b0, Nc = N, evc = ev;
        const uint64_t plc = pl;
        if (touched) {
            t = __builtin_ctzll(touched);
            b0 = __builtin_amdgcn_readfirstlane(m.bstart[t]);
            N = __builtin_amdgcn_readfirstlane(m.bstart[t + 1]) - b0;
            ev = lane < N ? m.bev[b0 + lane] : 0;
            pl = lane < N && N <= 64 ? (m.wide ? pb.poss[ev] : m.pl[b0 + lane]) : 0ull;
        }
        if (Nc == 0) continue;
        if (Nc <= 64) {
            const uint32_t r = wave_match_slot(R, Nc, plc, lane);
            if (lane < Nc) m.rr[evc] = (uint8_t)r;
        } else if (Nc <= kMaxSlotEvents) {
            if (lane == 0) {                    // rare: one lane, no barrier (the waves' slots differ)
                uint64_t* spl = m.wide ? m.pl + w * kMaxSlotEvents : m.pl + bc;   // wide: the wave's slot state
                uint8_t* smr = m.wide ? m.mr + w * kMaxSlotEvents : m.mr + bc;
                uint8_t* srm = m.wide ? m.rm + w * R : m.rm + tc * R;
                uint8_t* sdr = m.wide ? m.dr + w * R : m.dr + tc * R;
                if (m.wide)
                    for (int i = 0; i < Nc; ++i) spl[i] = pb.poss[m.bev[bc + i]];
                match_slot<4>(R, m.bev + bc, spl, Nc, smr, srm, sdr, m.rr);
            }
        } else {
            for (int i = lane; i < Nc; i += 64) m.rr[m.bev[bc + i]] = 0xFF;
            if (lane == 0) atomicOr(pb.status, 1);
        }
    }
#else
    if (lane < kSlots && ((touched >> lane) & 1ull)) {
        const int b0 = m.bstart[lane];
        const int N = m.bstart[lane + 1] - b0;
        const int R = pb.R;
        if (N > 0) {
            if (TT_MATCH_REG && N <= 32 && R <= 16)
                match_slot_reg(m.bev + b0, m.pl + b0, N, m.dr + lane * R, m.rr);
            else if (N <= 64)
                match_slot<1>(R, m.bev + b0, m.pl + b0, N, m.mr + b0, m.rm + lane * R, m.dr + lane * R, m.rr);
            else if (N <= kMaxSlotEvents)
                match_slot<4>(R, m.bev + b0, m.pl + b0, N, m.mr + b0, m.rm + lane * R, m.dr + lane * R, m.rr);
            else {
                for (int i = 0; i < N; ++i) m.rr[m.bev[b0 + i]] = 0xFF;
                atomicOr(pb.status, 1);
            }
        }
    }
#endif
    __syncthreads();
}

}  // namespace ttga

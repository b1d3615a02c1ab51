// Batched Solution::localSearch (Solution.cpp:471-769): one WAVE per
// individual, every individual with its own Park-Miller stream, bit-exact with
// the reference (same RNG draws, same first-improvement acceptance, same step
// budget shared by both phases).
//
// State of an individual, in LDS: slot and room of every event, per-slot event
// bitsets B[t] (the ascending timeslot_events lists), the room histogram of
// every slot and its room-clash pair count. A trial move (Move1/2/3,
// Solution.cpp:357-439) is never materialised as a copied Solution: the
// neighbour is the current state plus <=3 moved events; its <=3 touched slots
// get new bitsets NB[k] and are re-matched IN PARALLEL, one lane per slot
// (the assignRooms replay of tt_match.h), writing the neighbour's rooms into a
// mirror row nrr[]. The delta evaluators then read:
//   eventAffectedHcv(e)        = roomPairs(slot) + popcount(corr(e) & set) - corr(e,e)
//   affectedRoomInTimeslotHcv  = roomPairs(slot)
//   eventHcv(e)                = hist[slot][room(e)] - 1 + popcount(corr(e) & B) - corr(e,e)
//   eventScv / singleClassesScv from each student's 45-bit attendance mask
//                                (lanes = students of e, Solution.cpp:248-355)
// Accept copies the touched slots into the current state; reject restores nrr.
#include "tt_internal.h"
#include "tt_match.h"

namespace ttga {

constexpr int kLsTasks = 3;
// Two launches per call: the first sizes each of the 3 matcher tasks for 64
// events per slot (8 KB of LDS per wave at E = 400 instead of 14.6 KB, so about
// twice the waves per CU); an individual whose trial puts more than 64 events
// into a touched slot stops there, untouched in HBM, and is redone from its
// input by the second launch with tasks sized for kMaxSlotEvents.
constexpr int kLsCapSmall = 64;


// Profiling build (-DTT_LS_PROF, `make libttga_prof.so`, tools/ls_prof.py):
// per-section shader-clock totals of every wave, summed into g_ls_prof.
#ifdef TT_LS_PROF
enum { kPfInit, kPfBuild, kPfMatch, kPfCorr, kPfScv, kPfSync, kPfFeas, kPfTotal, kPfTrials, kPfVisits, kPfWaves, kPfScramble, kPfMatchCalls, kPfMatchEvents, kPfMatchSteps, kPfQ1, kPfQ1c, kPfQ1m, kPfQ2, kPfQ2c, kPfQ2m, kPfP1m2, kPfP1m2lb, kPfP1m1m, kPfP1m1a, kPfP1m1k, kPfVis1, kPfM1p1, kPfM2p1, kPfPh1, kPfPh2, kPfVis2, kPfM1p2, kPfM2p2, kPfSkip1, kPfHot1, kPfMaxTotal, kPfB1, kPfB2, kPfBInit, kPfP1m2r0, kPfP1m2a, kPfN };
__device__ unsigned long long g_ls_prof[kPfN];
// per individual of the first kLsWaveRec (tools/ls_tail.py): start and end of its wave
// (s_memrealtime, 100 MHz), its shader cycles and its full trials
constexpr int kLsWaveRec = 65536;
__device__ unsigned long long g_ls_wave[4 * kLsWaveRec];
#define LSP_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define LSP_ADD(St, i, v) ((St).prof[i] += __builtin_amdgcn_s_memtime() - (v))
#define LSP_CNT(St, i) ((St).prof[i] += 1)
#define LSP_SET(v) ((v) = __builtin_amdgcn_s_memtime())
#else
#define LSP_SET(v)
#define LSP_T(v)
#define LSP_ADD(St, i, v)
#define LSP_CNT(St, i)
#endif

// TT_LS_SLP (default 0): slp[p] = slot of the event at scramble position p and
// pos[e] = position of event e, kept with every accepted move, so a trial
// window reads a partner's event and its slot in one LDS round trip instead
// of two dependent ones. Same-box A/B (profiles/r03_s2_ab.json): +6 % on the
// comp01 local search (phase 1 and 2), -2 % on med phase 2; off.
#ifndef TT_LS_SLP
#define TT_LS_SLP 0
#endif

struct LsLayout {
    size_t sl, rr, nrr, evl, B, NB, rp, hist, misc, task, slp, pos, ps, sm, sinf;
    size_t task_bytes;
    size_t scratch;      // the task region: kLsTasks tasks, or the summaries' owner table if larger
    int NT;              // events per matcher task (min(E, 256))
    size_t bytes;
};

// TT_LS_POSS16: every event's possibleRooms mask copied into LDS as u16 when
// R <= 16 (0.8 KB per wave at E = 400), so a matcher task's masks and the
// phase-2 augmenting-path test read LDS instead of waiting on L2. Same-box A/B
// (profiles/r03_s11_ab.json): comp01 phase 1 -3 %, med phase 2 +5 % (one fewer
// wave per CU); off
#ifndef TT_LS_POSS16
#define TT_LS_POSS16 0
#endif
// TT_LS_SMASK: in phase 2 the state is feasible, so no student has two events
// in one slot and a student's 45-bit attendance mask changes by clearing the old
// and setting the new slot of a moved event. The masks of all students are kept
// in LDS for phase 2 (S <= 512), and eventScv / singleClassesScv read a student's
// mask instead of rebuilding it from the student's event list. The host turns
// them on (smS = S) only where the S*8 bytes of LDS cost no resident waves
// (ls_mask_students): same-box A/B at pop 4,096 / 8,192 (profiles/r03_s13_ab.json)
// med phase-2 LS(1000) -9 % (16 waves per CU fit either way), comp01 and lg +12..18 %
// (a second round of waves); at pop 65,536 (profiles/r03_s14_ab.json) forced masks
// gave med -2 %, comp01 +18 %, lg +33 %.
#ifndef TT_LS_SMASK
#define TT_LS_SMASK 1
#endif
constexpr size_t kSmaskMaxBytes = 4096;
// phase-2 share of an earlier call's steps above which the masks are worth resident waves
#ifndef TT_LS_MASK_SHARE
#define TT_LS_MASK_SHARE 0.5
#endif
// TT_LS_P1B: phase-1 room-pair lower bounds (below, SlotInfo) from a summary
// of a maximum matching of every slot (45 x 20 B per wave + 128 B scratch).
#ifndef TT_LS_P1B
#define TT_LS_P1B 1
#endif
// (R <= 16: the room sets fit 16 bits, a summary 8 bytes)
struct SlotInfo {
    uint16_t used;       // rooms matched in a maximum matching of the slot
    uint16_t fr;         // rooms from which an alternating path reaches a free room (free rooms included)
    int32_t nz;          // N << 16 | Z (events; events without a possible room), bit 31: trusted
};
constexpr int kP1bMaxRooms = 16;
// SlotInfo[45] of the slots, then [3] of the matcher tasks: 384 B per wave, in the
// phase-2 student-mask region when there is one (the two phases never overlap)
constexpr size_t kSinfBytes = sizeof(SlotInfo) * (kSlots + 3);
// A matcher task: ev [NT] u16 and hist [R] u16 (the wave matcher's), then, only
// where a slot of more than 64 events can reach the lane-serial matcher (NT > 64),
// its pl [NT] u64, mr [NT], rm [R] and dr [R]. TT_LS_TASK_COMPACT = 0 allocates
// the serial matcher's arrays in every launch (the round-4 layout's size: 11 NT +
// 4 R bytes per task, against 2 NT + 2 R; at E >= 64 the first launch's three
// tasks take 2.3 KB of a wave's LDS instead of 0.5 KB).
#ifndef TT_LS_TASK_COMPACT
#define TT_LS_TASK_COMPACT 1
#endif
__host__ __device__ inline size_t task_off_pl(int NT, int R) { return (2 * (size_t)NT + 2 * (size_t)R + 7) & ~(size_t)7; }
// cap: events per matcher task (kLsCapSmall for the first launch, kMaxSlotEvents for the redo launch)
// S: students with phase-2 masks (0: none)
__host__ __device__ inline LsLayout ls_layout(int E, int R, int EW, int cap, int S) {
    LsLayout L;
    size_t b = 0;
    auto al = [&](size_t a) { b = (b + a - 1) & ~(a - 1); };
    L.sl = b; b += E + 1;
    L.rr = b; b += E;
    L.nrr = b; b += E;
    al(2); L.evl = b; b += 2 * (size_t)E;
#if TT_LS_SLP
    L.pos = b; b += 2 * (size_t)E;
    L.slp = b; b += (size_t)E;
#else
    L.pos = L.slp = 0;
#endif
#if TT_LS_POSS16
    L.ps = b; if (R <= 16) b += 2 * (size_t)E;        // possibleRooms as u16 (R <= 16)
#else
    L.ps = 0;
#endif
    al(8);
#if TT_LS_SMASK
    L.sm = b; if (S > 0 && 8 * (size_t)S <= kSmaskMaxBytes) b += 8 * (size_t)S;   // phase-2 student masks (S = smS)
#else
    L.sm = 0;
#endif
    L.B = b; b += 8 * (size_t)kSlots * EW;
    L.NB = b; b += 8 * (size_t)kLsTasks * EW;
    L.rp = b; b += 4 * (size_t)kSlots;
    L.hist = b; b += 2 * (size_t)kSlots * R;
    // phase-1 slot summaries: aliased with the phase-2 student masks when those exist
    L.sinf = 0;
    if (TT_LS_P1B && R <= kP1bMaxRooms) {
        if (L.sm && S > 0 && 8 * (size_t)S <= kSmaskMaxBytes && 8 * (size_t)S >= kSinfBytes) L.sinf = L.sm;
        else { al(8); L.sinf = b; b += kSinfBytes; }
    }
    al(4); L.misc = b; b += 4 * 32;
    L.NT = E < cap ? E : cap;
    L.task_bytes = (task_off_pl(L.NT, R) + (L.NT > 64 || !TT_LS_TASK_COMPACT ? 9 * (size_t)L.NT + 2 * (size_t)R : 0) + 15) &
                   ~(size_t)15;
    al(16); L.task = b;
    L.scratch = kLsTasks * L.task_bytes;
    // the phase-1 summaries' start-up owner table [45][R] u16 shares the task region
    if (L.sinf && 2 * (size_t)kSlots * R > L.scratch) L.scratch = (2 * (size_t)kSlots * R + 15) & ~(size_t)15;
    b += L.scratch;
    L.bytes = (b + 15) & ~(size_t)15;
    return L;
}

struct LsTask {
    uint64_t* pl;
    uint16_t* ev;
    uint8_t* mr;
    uint8_t* rm;
    uint8_t* dr;
    uint16_t* hist;
};

struct LsState;
__device__ __forceinline__ LsTask get_task(const LsState& S, int k);

struct LsState {
    DevProblem pb;
    int E, R, EW, lane;
    uint8_t *sl, *rr, *nrr;
    uint16_t* evl;
    uint16_t* pos;       // [E] position of each event in evl (TT_LS_SLP)
    uint8_t* slp;        // [E] slot of the event at each position (TT_LS_SLP)
    uint64_t *B, *NB;
    const uint16_t* ps;  // [E] possibleRooms in LDS (R <= 16), else null (TT_LS_POSS16)
    uint64_t* sm;        // [S] phase-2 attendance masks (TT_LS_SMASK), null outside phase 2
    int32_t* rp;
    uint16_t* hist;
    int32_t* misc;       // [0..2] neighbour room pairs per task, [3] redo flag, [4..6] events per task
    uint8_t* task_base;
    int task_bytes, NT, scratch;
    // neighbour description (wave-uniform)
    int nmv, mv_e[3], mv_t[3];
    int nts, ts[3];
    // Move1 loops: the old slot minus the moved event (task 1) is the same set
    // for every target slot, so its matching is kept from one rejected trial
    // to the next (c1_valid) instead of being recomputed
    int c1_valid;
    int listed;          // task event lists built for the current neighbour
    // phase 2: the state stays feasible, so every slot's rooms are distinct and
    // hist[] is reused as the owner table oe[slot * R + room] (event, 0xFFFF free)
    int phase2;
    // phase-1 pair bounds (TT_LS_P1B): per-slot matching summaries; null sinf: off.
    // one base pointer: sinf[45] of the slots, then tsi[3] of the matcher tasks
    SlotInfo* sinf;
    int tvalid;          // bit k: tsi[k] describes the current neighbour's task k
#ifdef TT_LS_PROF
    uint64_t prof[kPfN];
#endif
};

__device__ __forceinline__ SlotInfo* tsi_of(const LsState& S) { return S.sinf + kSlots; }

__device__ __forceinline__ LsTask get_task(const LsState& S, int k) {
    uint8_t* tb = S.task_base + (size_t)k * S.task_bytes;
    LsTask T;
    T.ev = (uint16_t*)tb;
    T.hist = T.ev + S.NT;
    T.pl = (uint64_t*)(tb + task_off_pl(S.NT, S.R));      // lane-serial matcher only (NT > 64)
    T.mr = (uint8_t*)(T.pl + S.NT);
    T.rm = T.mr + S.NT;
    T.dr = T.rm + S.R;
    return T;
}

__device__ __forceinline__ uint64_t poss_of(const LsState& S, int e) {
    return S.ps ? (uint64_t)S.ps[e] : S.pb.poss[e];
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int slot_nb(const LsState& S, int j) {
    int s = S.sl[j];
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (k < S.nmv && j == S.mv_e[k]) s = S.mv_t[k];
    return s;
}

// sum over words of popcount(corr64[e] & set[w]) - corr(e,e)  (the "i != e" of the reference)
__device__ __forceinline__ int corr_in_set(LsState& S, int e, const uint64_t* set) {
    LSP_T(t0);
    int c = 0;
    for (int w = S.lane; w < S.EW; w += 64) c += __popcll(S.pb.corr64[(size_t)e * S.EW + w] & set[w]);
    c = wave_sum(c);
    const int self = (int)((S.pb.corr64[(size_t)e * S.EW + (e >> 6)] >> (e & 63)) & 1ull);
    LSP_ADD(S, kPfCorr, t0);
    return c - self;
}

// TT_LS_ROWB: a lane's own correlation row (corr64[e], EW words in L2) against an
// LDS word set, loaded 8 words at a time with all 8 loads in flight before the
// first is used -- the plain word loop waited out one L2 round trip per word
// (EW of them per row; 49 per whole-population pass at E = 400).
#ifndef TT_LS_ROWB
#define TT_LS_ROWB 1
#endif
// sum over w < EW of popcount(row[w] & set[w]) minus the row's own bit e
__device__ __forceinline__ int row_pop_in(const uint64_t* __restrict__ row, const uint64_t* set, int EW, int e) {
    int c = 0;
#if TT_LS_ROWB
    for (int w0 = 0; w0 < EW; w0 += 8) {
        uint64_t x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = w0 + k < EW ? row[w0 + k] : 0ull;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            c += __popcll(x[k] & (w0 + k < EW ? set[w0 + k] : 0ull));
            if (w0 + k == (e >> 6)) c -= (int)((x[k] >> (e & 63)) & 1ull);
        }
    }
#else
    for (int w = 0; w < EW; ++w) c += __popcll(row[w] & set[w]);
    c -= (int)((row[e >> 6] >> (e & 63)) & 1ull);
#endif
    return c;
}

// eventAffectedHcv(e) (Solution.cpp:194-215) in the current state
__device__ __forceinline__ int eah_cur(LsState& S, int e) {
    const int t = S.sl[e];
    return S.rp[t] + corr_in_set(S, e, S.B + (size_t)t * S.EW);
}

__device__ __forceinline__ int task_of(const LsState& S, int t) {
    int k = 0;
#pragma unroll
    for (int q = 0; q < 3; ++q)
        if (q < S.nts && S.ts[q] == t) k = q;
    return k;
}

// eventAffectedHcv(e) in the neighbour
__device__ __forceinline__ int eah_nb(LsState& S, int e) {
    const int k = task_of(S, slot_nb(S, e));
    return S.misc[k] + corr_in_set(S, e, S.NB + (size_t)k * S.EW);
}

// the correlation part of eventAffectedHcv(e) in the neighbour (needs NB, not rooms)
__device__ __forceinline__ int corr_nb(LsState& S, int e) {
    return corr_in_set(S, e, S.NB + (size_t)task_of(S, slot_nb(S, e)) * S.EW);
}

// eventHcv(e) (Solution.cpp:173-191) in the current state
__device__ __forceinline__ int ehcv_cur(LsState& S, int e) {
    const int t = S.sl[e];
    return (int)S.hist[t * S.R + S.rr[e]] - 1 + corr_in_set(S, e, S.B + (size_t)t * S.EW);
}

// eventScv(e) and singleClassesScv(e) (Solution.cpp:248-355) in the current
// (nb = false) or neighbour (nb = true) state.
// student st attends event q (its padded event list holds q)
__device__ __forceinline__ bool attends(const DevProblem& pb, int st, int q) {
    bool f = false;
    const int c0 = pb.stc_off[st], c1 = pb.stc_off[st + 1];
    for (int c = c0; c < c1; c += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f |= pb.stc_ev[c + j] == q;
    }
    return f;
}

__device__ __forceinline__ void scv_terms(LsState& S, int e, bool nb, int& es, int& scs) {
    LSP_T(t0);
    const DevProblem& pb = S.pb;
    const int t = nb ? slot_nb(S, e) : S.sl[e];
    const int day = t / 9, pos = t - 9 * day;
    const int k0 = pb.ev_off[e], k1 = pb.ev_off[e + 1];
    int a = 0, b = 0;
    // phase-2 masks: the neighbour's mask of a student of e clears the old and sets the
    // new slot of every moved event the student attends -- e itself, and any other moved
    // event correlated with e (a shared student); clears before sets (a swap keeps both)
    int oth = 0;                                       // bit q: moved event q != e correlated with e
    if (S.sm && nb) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            if (q >= S.nmv) break;
            const int qe = S.mv_e[q];
            if (qe != e && ((pb.corr64[(size_t)e * S.EW + (qe >> 6)] >> (qe & 63)) & 1ull)) oth |= 1 << q;
        }
    }
    for (int k = k0 + S.lane; k < k1; k += 64) {
        const int st = pb.ev_stu[k];
        uint64_t m = 0;
        if (S.sm) {
            m = S.sm[st];
            if (nb) {
                uint64_t clr = 1ull << S.sl[e], set = 1ull << t;
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    if (!((oth >> q) & 1)) continue;
                    const int qe = S.mv_e[q];
                    if (attends(pb, st, qe)) { clr |= 1ull << S.sl[qe]; set |= 1ull << S.mv_t[q]; }
                }
                m = (m & ~clr) | set;
            }
        } else {
            const int c0 = pb.stc_off[st], c1 = pb.stc_off[st + 1];
            for (int c = c0; c < c1; c += 8) {
                int ev[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) ev[j] = pb.stc_ev[c + j];
#pragma unroll
                for (int j = 0; j < 8; ++j) m |= 1ull << ((nb ? slot_nb(S, ev[j]) : S.sl[ev[j]]) & 63);
            }
        }
        const uint32_t dm = (uint32_t)(m >> (9 * day)) & 0x1FFu;
        const uint32_t others = dm & ~(1u << pos);
        auto at = [&](int x) -> int { return (int)((dm >> x) & 1u); };
        if (pos < 8 && at(pos + 1)) a += (pos < 7 ? at(pos + 2) : 0) + (pos > 0 ? at(pos - 1) : 0);
        if (pos > 1) a += at(pos - 1) & at(pos - 2);
        a += others == 0u;
        b += __popc(others) == 1;
    }
    es = wave_sum(a) + (pos == 8 ? pb.sn[e] : 0);
    scs = wave_sum(b);
    LSP_ADD(S, kPfScv, t0);
}

// TT_LS_DISC_ALL: the room stage's discovering-room ballot over all room lanes,
// masked by the uniform M afterwards (no per-lane M test).
#ifndef TT_LS_DISC_ALL
#define TT_LS_DISC_ALL 1
#endif
// TT_LS_WLT: the matcher's room transpose by v_writelane instead of a
// compare-and-select per room.
#ifndef TT_LS_WLT
#define TT_LS_WLT 1
#endif
// (writelane64 is in tt_match.h; nothing else in the local-search kernel uses
// M0 -- no LDS-DMA, no movrel.)

// Wave matcher for one touched slot of N <= 64 events, the same search as
// match_slot<1> (tt_match.h, Solution.cpp:772-891), with its state in
// registers: lane i holds event i's possible-room mask (pl) and matched room
// (mr); lane j holds room j's matched event (rm), search dad (dr) and the mask
// of the slot's events that may use it (ev_of_room); the seen/fringe sets are
// wave-uniform (scalar) bitsets. The search expands every fringe event before
// any room, so its first stage -- all unmatched events in ascending order --
// is closed-form: the rooms seen are those with an unmatched candidate event,
// and room j's dad is the lowest unmatched event that may use it. Only the
// room stage (ascending rooms, a matched room's event expanded at once) walks
// step by step.
__device__ __forceinline__ void match_task_wave(LsState& S, int k, int N, int ev, uint64_t pl) {
    LSP_T(t0);
    LSP_CNT(S, kPfMatchCalls);
#ifdef TT_LS_PROF
    S.prof[kPfMatchEvents] += N;
#endif
    const int lane = S.lane, R = S.R;
    constexpr uint32_t NONE = 0xFFu;
    const bool act = lane < N;
    const uint32_t pl_lo = (uint32_t)pl, pl_hi = (uint32_t)(pl >> 32);
    // transpose: ev_of_room (lane j) = the events whose possible rooms include j:
    // one ballot per room, written into lane j by v_writelane; pl is zero past the
    // N events (load_tasks)
#if TT_LS_WLT
    uint32_t eor_lo = 0, eor_hi = 0;
    {
        const int r1 = R < 32 ? R : 32;
        for (int j = 0; j < r1; ++j) writelane64(eor_lo, eor_hi, ballot((pl_lo >> j) & 1u), j);
        for (int j = 32; j < R; ++j) writelane64(eor_lo, eor_hi, ballot((pl_hi >> (j - 32)) & 1u), j);
    }
    const uint64_t eor = ((uint64_t)eor_hi << 32) | eor_lo;
#else
    uint64_t eor = 0;
    for (int j0 = 0; j0 < R; j0 += 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t b = ballot((pl >> (j0 + q)) & 1ull);
            if (lane == j0 + q) eor = b;
        }
    }
#endif
    // lane j also keeps the possible rooms of its matched event (plr), so a
    // search step reads rm and plr at the same lane j: no dependent readlane
    uint32_t mr = NONE, rm = 0, dr = 0, plr_lo = 0, plr_hi = 0;
    uint64_t unm = N >= 64 ? ~0ull : ((1ull << N) - 1ull);
    uint64_t rmatched = 0;
    for (;;) {
        // stage 1 (closed form): expand all unmatched events, ascending
        const uint64_t cand = eor & unm;
        uint64_t sr = ballot(cand != 0ull), fr = sr;          // eor is zero on lanes >= R (no room bit there)
        if (cand) dr = (uint32_t)__builtin_ctzll(cand);
        // stage 2: fringe rooms ascending; a matched room's event is expanded at
        // once. Each room enters the fringe once and each matched event is
        // reached only through its own room (already seen), so neither a seen-
        // event test nor the event's own room needs masking.
        // Bulk form of the ascending walk: every fringe room below the lowest
        // free one is matched, and popping a room whose event reaches no unseen
        // room changes nothing but the fringe, so all such rooms up to the first
        // one that does discover rooms (one ballot over the room lanes) are
        // popped at once; that room is expanded as in the step-by-step walk.
        int sink = -1;
        for (;;) {
            const uint64_t freef = fr & ~rmatched;
            const uint64_t M = fr & (freef ? (freef & (0ull - freef)) - 1ull : ~0ull);
            const uint64_t plr = ((uint64_t)plr_hi << 32) | plr_lo;
#if TT_LS_DISC_ALL
            const uint64_t disc = ballot((plr & ~sr) != 0ull) & M;      // M is uniform: mask after the ballot
#else
            const uint64_t disc = ballot(((M >> lane) & 1ull) && (plr & ~sr) != 0ull);
#endif
            LSP_CNT(S, kPfMatchSteps);
            if (!disc) {                                   // the walk reaches the lowest free room
                if (freef) sink = __builtin_ctzll(freef);
                break;
            }
            const int j = __builtin_ctzll(disc);
            fr &= ~(M & ((2ull << j) - 1ull));             // pops M's rooms up to j (j <= 63)
            const int i2 = __builtin_amdgcn_readlane((int)rm, j);
            const uint64_t pli = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)plr_hi, j) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)plr_lo, j);
            const uint64_t nr = pli & ~sr;
            sr |= nr;
            fr |= nr;
            if ((nr >> lane) & 1ull) dr = (uint32_t)i2;
        }
        if (sink < 0) break;
        // maxMatching augmentation (Solution.cpp:836-849)
        int j = sink;
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
    const bool un = act && mr == NONE;
    const uint64_t unb = ballot(un);
    uint32_t r = mr;
    if (unb) {                                     // wave-uniform: usually every event is placed
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
        r = !un ? mr : (pl ? v : (below ? carried : 0u));
    }
    // room histogram (lane j = room j) and the pairs of events sharing a room
    // (r < R for every event): matched events hold distinct rooms, the rooms in
    // rmatched, so only the unplaced events add to a room's count and make pairs
    const LsTask T = get_task(S, k);
    uint32_t cnt_r = (uint32_t)((rmatched >> lane) & 1ull);
    int pr = 0;
    for (uint64_t um = unb; um; um &= um - 1) {
        const int i = __builtin_ctzll(um);
        const int ri = __builtin_amdgcn_readlane((int)r, i);
        pr += __builtin_amdgcn_readlane((int)cnt_r, ri);
        if (lane == ri) ++cnt_r;
    }
    if (act) S.nrr[ev] = (uint8_t)r;
    if (lane < R) T.hist[lane] = (uint16_t)cnt_r;
    if (lane == 0) S.misc[k] = pr;
    if (S.sinf) {
        // phase-1 pair bounds: this maximum matching's summary (see SlotInfo), read off
        // the registers -- room lane j: its matched event's possible rooms (plr)
        const bool mj = (rmatched >> lane) & 1ull;
        const uint64_t plr = ((uint64_t)plr_hi << 32) | plr_lo;
        uint64_t fr = (R >= 64 ? ~0ull : ((1ull << R) - 1)) & ~rmatched;
        for (;;) {
            const uint64_t fn = fr | ballot(mj && (plr & fr) != 0ull);
            if (fn == fr) break;
            fr = fn;
        }
        const int z = __popcll(ballot(act && pl == 0ull));
        if (lane == 0) {
            tsi_of(S)[k].used = (uint16_t)rmatched;
            tsi_of(S)[k].fr = (uint16_t)fr;
            tsi_of(S)[k].nz = (int)0x80000000 | (N << 16) | z;
        }
        S.tvalid |= 1 << k;
    }
    LSP_ADD(S, kPfMatch, t0);
}

// Lane-serial matcher for a touched slot of 64 < N <= 256 events (one lane):
// rare, so out of line (TT_LS_SERIAL_CALL) -- inlined at each of match_tasks'
// call sites it made up much of the kernel's 166 KB of code. Returns the
// slot's room-clash pairs; the rooms go to nrr.
#ifndef TT_LS_TASK_LOOP
#define TT_LS_TASK_LOOP 1
#endif
#ifndef TT_LS_M1WIN
#define TT_LS_M1WIN 1
#endif
// visit rows one visit ahead: same-box A/B +2..+11 % (profiles/r03_s5_ab.json); off
#ifndef TT_LS_ROWPF
#define TT_LS_ROWPF 0
#endif
// With the phase-1 eventHcv flags a skip moves the visit index by several
// positions, so a row prefetched for position i+1 would belong to the wrong
// event: the two are exclusive.
#if TT_LS_ROWPF && (!defined(TT_LS_HOT) || TT_LS_HOT)
#error "TT_LS_ROWPF needs TT_LS_HOT=0 (a flag skip invalidates the prefetched row)"
#endif
#ifndef TT_LS_SERIAL_CALL
#define TT_LS_SERIAL_CALL 1
#endif
#if TT_LS_SERIAL_CALL
__device__ __noinline__
#else
__device__ __forceinline__
#endif
int match_task_serial(int R, int N, const uint64_t* poss, uint16_t* ev, uint64_t* pl, uint8_t* mr, uint8_t* rm,
                      uint8_t* dr, uint16_t* hist, uint8_t* nrr) {
    for (int i = 0; i < N; ++i) pl[i] = poss[ev[i]];
    for (int r = 0; r < R; ++r) hist[r] = 0;
    match_slot<4>(R, ev, pl, N, mr, rm, dr, nrr);
    int pairs = 0;
    for (int i = 0; i < N; ++i) {
        const int r = nrr[ev[i]];
        pairs += hist[r];
        hist[r] = (uint16_t)(hist[r] + 1);
    }
    return pairs;
}

// Builds NB[k] for the touched slots; lane k lists the events of slot k.
__device__ __forceinline__ void build_nb(LsState& S) {
    LSP_T(t0);
    LSP_CNT(S, kPfTrials);
    const int EW = S.EW;
    // static indices into ts/mv_e/mv_t (unrolled to 3): a runtime index would
    // force the whole LsState into scratch and every LDS pointer through flat loads
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (k >= S.nts) break;
        const int t = S.ts[k];
        for (int w = S.lane; w < EW; w += 64) {
            uint64_t x = S.B[(size_t)t * EW + w];
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int e = S.mv_e[q];
                if (q < S.nmv && S.sl[e] == t && (e >> 6) == w) x &= ~(1ull << (e & 63));
            }
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int e = S.mv_e[q];
                if (q < S.nmv && S.mv_t[q] == t && (e >> 6) == w) x |= 1ull << (e & 63);
            }
            S.NB[(size_t)k * EW + w] = x;
        }
    }
    S.listed = 0;
    wave_sync();
    LSP_ADD(S, kPfBuild, t0);
}

// Lists the events of each touched slot for the matcher (lane k lists slot k);
// done only for trials that reach a matching.
__device__ __forceinline__ void list_tasks(LsState& S) {
    LSP_T(t0);
    const int EW = S.EW;
    if (S.lane < S.nts) {
        const int k = S.lane;
        const LsTask T = get_task(S, k);
        const uint64_t* nb = S.NB + (size_t)k * EW;
        int N = 0;
        for (int w = 0; w < EW; ++w)
            for (uint64_t x = nb[w]; x; x &= x - 1) {
                if (N < S.NT) T.ev[N] = (uint16_t)(64 * w + __builtin_ctzll(x));
                ++N;
            }
        S.misc[4 + k] = N;
    }
    wave_sync();
    LSP_ADD(S, kPfBuild, t0);
}

// Re-matches the touched slots in kmask (after build_nb): the wave matcher runs
// the slots one after another (the lane-serial match_slot<4> for a slot of more
// than 64 events). Returns true when the first launch must redo the individual.
struct TaskRegs {
    int tn[3], tev[3];
    uint64_t tpl[3];
};

// TT_LS_TASK_LATE: a task's events and possible rooms are loaded in the task
// loop right before its matching, instead of all three tasks' at once ahead of
// the loop: the 12 VGPRs of the early form stay live across the inlined
// matcher, which at the kernel's 96 VGPRs spilled them to scratch (the largest
// group of the kernel's scratch accesses)
#ifndef TT_LS_TASK_LATE
#define TT_LS_TASK_LATE 1
#endif
// every task's events and possible rooms into registers at once (one L2 round
// trip), issued as early as the trial allows so the latency overlaps other work
__device__ __forceinline__ TaskRegs load_tasks(LsState& S, int kmask) {
    // task 1 kept from the previous rejected Move1 trial (set only inside a phase-1 Move1 loop)
    if (S.c1_valid && S.nts == 2) kmask &= ~2;
    if (!S.listed) {
        list_tasks(S);
        S.listed = 1;
    }
    TaskRegs r;
    if (TT_LS_TASK_LATE) {
#pragma unroll
        for (int k = 0; k < 3; ++k) { r.tn[k] = 0; r.tev[k] = 0; r.tpl[k] = 0ull; }
        return r;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        r.tn[k] = k < S.nts && ((kmask >> k) & 1) ? S.misc[4 + k] : 0;
        const bool a = S.lane < r.tn[k] && r.tn[k] <= 64;
        r.tev[k] = a ? get_task(S, k).ev[S.lane] : 0;
        r.tpl[k] = a ? poss_of(S, r.tev[k]) : 0ull;
    }
    return r;
}

__device__ __forceinline__ bool match_tasks(LsState& S, int kmask, const TaskRegs& tr) {
    if (S.c1_valid && S.nts == 2) kmask &= ~2;
    if (!(kmask & ((1 << S.nts) - 1))) return false;            // nothing to match: no sync
    LSP_T(t0);
    // TT_LS_TASK_LOOP: the task loop stays a loop (one inlined matcher per call
    // site instead of three); the task's registers are picked by selects
#if TT_LS_TASK_LOOP
#pragma unroll 1
#else
#pragma unroll
#endif
    for (int k = 0; k < 3; ++k) {
        if (k >= S.nts) break;
        if (!((kmask >> k) & 1)) continue;
        int N, tevk;
        uint64_t tplk;
        if (TT_LS_TASK_LATE) {
            N = __builtin_amdgcn_readfirstlane(S.misc[4 + k]);
            const bool a = S.lane < N && N <= 64;
            tevk = a ? get_task(S, k).ev[S.lane] : 0;
            tplk = a ? poss_of(S, tevk) : 0ull;
        } else {
            N = k == 0 ? tr.tn[0] : k == 1 ? tr.tn[1] : tr.tn[2];
            tevk = k == 0 ? tr.tev[0] : k == 1 ? tr.tev[1] : tr.tev[2];
            tplk = k == 0 ? tr.tpl[0] : k == 1 ? tr.tpl[1] : tr.tpl[2];
        }
        if (N > S.NT) {                                             // task capacity exceeded
            if (S.lane == 0) {
                if (S.NT < kMaxSlotEvents && S.NT < S.E) {
                    S.misc[3] = 1;                                  // first launch: redo with full tasks
                } else {
                    atomicOr(S.pb.status, 1);
                    const LsTask T = get_task(S, k);
                    for (int i = 0; i < S.NT; ++i) S.nrr[T.ev[i]] = 0xFF;
                    S.misc[k] = 0;
                }
            }
            wave_sync();
            if (S.misc[3]) break;
        } else if (N == 0) {
            if (S.lane == 0) S.misc[k] = 0;
        } else if (N <= 64) {
            match_task_wave(S, k, N, tevk, tplk);
        } else {                                                    // 64 < N <= 256: lane-serial matcher
            if (S.lane == 0) {
                const LsTask T = get_task(S, k);
                S.misc[k] = match_task_serial(S.R, N, S.pb.poss, T.ev, T.pl, T.mr, T.rm, T.dr, T.hist, S.nrr);
            }
            S.tvalid &= ~(1 << k);                                  // accept rebuilds this slot's summary
            wave_sync();
        }
    }
    wave_sync();
    LSP_ADD(S, kPfBuild, t0);
    return S.misc[3] != 0;
}

__device__ __forceinline__ bool match_tasks(LsState& S, int kmask) {
    if (S.c1_valid && S.nts == 2) kmask &= ~2;
    if (!(kmask & ((1 << S.nts) - 1))) return false;            // nothing to match: no listing, no loads
    return match_tasks(S, kmask, load_tasks(S, kmask));
}

__device__ __forceinline__ bool build_and_match(LsState& S) {
    build_nb(S);
    return match_tasks(S, 7);
}

// events of neighbour slot k: copy rooms between rr and nrr
__device__ __forceinline__ void sync_rooms(LsState& S, bool accept) {
    LSP_T(t0);
    for (int k = 0; k < S.nts; ++k) {
        const uint64_t* nb = S.NB + (size_t)k * S.EW;
        for (int w = S.lane; w < S.EW; w += 64) {
            uint64_t x = nb[w];
            while (x) {
                const int e = 64 * w + __builtin_ctzll(x);
                x &= x - 1;
                if (accept) S.rr[e] = S.nrr[e];
                else S.nrr[e] = S.rr[e];
            }
        }
    }
    wave_sync();
    LSP_ADD(S, kPfSync, t0);
}

// nrr = rr for the events of neighbour slot K
template <int K>
__device__ __forceinline__ void restore_task(LsState& S) {
    const uint64_t* nb = S.NB + (size_t)K * S.EW;
    for (int w = S.lane; w < S.EW; w += 64)
        for (uint64_t x = nb[w]; x; x &= x - 1) {
            const int e = 64 * w + __builtin_ctzll(x);
            S.nrr[e] = S.rr[e];
        }
    wave_sync();
}

// Rejected Move1 trial. A two-slot neighbour (target t, then the old slot)
// keeps task 1 -- the old slot minus the moved event, the same set for every
// target -- matched in nrr, NB[1], hist and misc[1] for the next trial.
__device__ __forceinline__ void reject_move1(LsState& S) {
    if (S.nts == 2) {
        restore_task<0>(S);
        S.c1_valid = 1;
    } else {                          // t == old slot: everything re-matched, drop the kept task
        sync_rooms(S, false);
        S.c1_valid = 0;
    }
}

// end of a Move1 loop: restore the kept task
__device__ __forceinline__ void cache_drop(LsState& S) {
    if (S.c1_valid) {
        restore_task<1>(S);
        S.c1_valid = 0;
    }
}

__device__ __forceinline__ void sinf_build(LsState& S, int t);
__device__ __forceinline__ void accept(LsState& S) {
    LSP_T(t0);
    S.c1_valid = 0;
    if (S.sm) {                       // phase-2 masks: clear every moved event's old slot, then set the new ones
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            if (q >= S.nmv) break;
            const int qe = S.mv_e[q];
            const uint64_t c = ~(1ull << S.sl[qe]);
            for (int k = S.pb.ev_off[qe] + S.lane; k < S.pb.ev_off[qe + 1]; k += 64) S.sm[S.pb.ev_stu[k]] &= c;
        }
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            if (q >= S.nmv) break;
            const int qe = S.mv_e[q];
            const uint64_t st_bit = 1ull << S.mv_t[q];
            for (int k = S.pb.ev_off[qe] + S.lane; k < S.pb.ev_off[qe + 1]; k += 64) S.sm[S.pb.ev_stu[k]] |= st_bit;
        }
    }
    sync_rooms(S, true);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (k >= S.nts) break;
        const int t = S.ts[k];
        for (int w = S.lane; w < S.EW; w += 64) S.B[(size_t)t * S.EW + w] = S.NB[(size_t)k * S.EW + w];
        const LsTask T = get_task(S, k);
        for (int r = S.lane; r < S.R; r += 64) S.hist[t * S.R + r] = S.phase2 ? (uint16_t)0xFFFF : T.hist[r];
    }
    if (S.phase2) {                   // owner table rows of the touched slots, from the new rooms
        wave_sync();
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k >= S.nts) break;
            const int t = S.ts[k];
            for (int w = S.lane; w < S.EW; w += 64)
                for (uint64_t x = S.NB[(size_t)k * S.EW + w]; x; x &= x - 1) {
                    const int e = 64 * w + __builtin_ctzll(x);
                    S.hist[t * S.R + S.rr[e]] = (uint16_t)e;
                }
        }
    }
    if (S.lane == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k)
            if (k < S.nts) S.rp[S.ts[k]] = S.misc[k];
#pragma unroll
        for (int q = 0; q < 3; ++q)
            if (q < S.nmv) {
                S.sl[S.mv_e[q]] = (uint8_t)S.mv_t[q];
#if TT_LS_SLP
                S.slp[S.pos[S.mv_e[q]]] = (uint8_t)S.mv_t[q];
#endif
            }
    }
    wave_sync();
    if (S.sinf) {                     // phase-1 pair bounds: the re-matched slots' summaries (reference rooms)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k >= S.nts) break;
            if ((S.tvalid >> k) & 1) {                     // from the wave matcher's own result
                if (S.lane == 0) S.sinf[S.ts[k]] = tsi_of(S)[k];
            } else {
                sinf_build(S, S.ts[k]);
            }
        }
        wave_sync();
    }
    LSP_ADD(S, kPfSync, t0);
}

__device__ __forceinline__ void add_touched(LsState& S, int t) {
    const bool seen = (S.nts > 0 && S.ts[0] == t) || (S.nts > 1 && S.ts[1] == t) || (S.nts > 2 && S.ts[2] == t);
    if (seen) return;
    if (S.nts == 0) S.ts[0] = t;
    else if (S.nts == 1) S.ts[1] = t;
    else S.ts[2] = t;
    S.nts++;
}

__device__ __forceinline__ void set_move(LsState& S, int type, int e1, int a2, int e3) {
    // type 1: e1 -> slot a2; type 2: swap e1, a2; type 3: e1->slot(a2), a2->slot(e3), e3->slot(e1)
    S.nts = 0;
    S.tvalid = S.c1_valid ? (S.tvalid & 2) : 0;             // a kept task 1 keeps its summary
    if (type == 1) {
        S.nmv = 1; S.mv_e[0] = e1; S.mv_t[0] = a2;
        add_touched(S, a2); add_touched(S, S.sl[e1]);
    } else if (type == 2) {
        const int t1 = S.sl[e1], t2 = S.sl[a2];
        S.nmv = 2; S.mv_e[0] = e1; S.mv_t[0] = t2; S.mv_e[1] = a2; S.mv_t[1] = t1;
        add_touched(S, t2); add_touched(S, t1);
    } else {
        const int t1 = S.sl[e1], t2 = S.sl[a2], t3 = S.sl[e3];
        S.nmv = 3; S.mv_e[0] = e1; S.mv_t[0] = t2; S.mv_e[1] = a2; S.mv_t[1] = t3; S.mv_e[2] = e3; S.mv_t[2] = t1;
        add_touched(S, t2); add_touched(S, t3); add_touched(S, t1);
    }
}

// whole-solution feasibility (Solution.cpp:63-84) from the incremental state
__device__ __forceinline__ bool feasible_now(LsState& S) {
    LSP_T(t0);
    int h = 0;
    for (int t = S.lane; t < kSlots; t += 64) h += S.rp[t];
    for (int k = 0; 64 * k < S.E; ++k) {                   // wave-uniform
        const int e = 64 * k + S.lane;
        if (e < S.E) {
            const int t = S.sl[e];
            const int c = row_pop_in(S.pb.corr64 + (size_t)e * S.EW, S.B + (size_t)t * S.EW, S.EW, e);
            h += c;   // every correlated same-slot pair is counted twice, only zero matters
            h += (int)(((S.pb.poss[e] >> S.rr[e]) & 1ull) ^ 1ull);
        }
    }
    const bool f = wave_sum(h) == 0;
    LSP_ADD(S, kPfFeas, t0);
    return f;
}

// ---- correlation shortcuts. Phase 1 (Solution.cpp:497-618): the visited
// event's row and X[t] give corr_nb(ei) of a Move1 to t and of a Move2 with an
// event of t without reading the row again; a Move2 partner's row is loaded
// once per trial (one trial ahead) and its two counts share one reduction, so
// the lower bound rejects most trials before any neighbour is built.
// Phase-2 shortcuts (Solution.cpp:619-768). In phase 2 the state is
// feasible and only moves with eventAffectedHcv == 0 for every moved event are
// accepted, so a trial is rejected, before any neighbour is built, when
//  * a moved event meets a correlated event in its new slot (the count of the
//    visited event's correlated events per slot, X[t], and the OR of its
//    slot-mates' correlation rows, Z, are computed once per visit), or
//  * a touched slot cannot be room-matched without a clash: the reference's
//    assignRooms gives zero clash pairs exactly when a perfect matching exists
//    (it is a maximum matching, and an unmatched event has no free possible
//    room), and a perfect one exists exactly when the moved-in event has an
//    augmenting path from the slot's current (clash-free) rooms.
// The RNG draws are the reference's; every other trial takes the full path.
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}
// bit e of a row held one 64-bit word per lane
__device__ __forceinline__ bool row_bit(uint64_t lane_words, int e) {
    return (readlane64(lane_words, e >> 6) >> (e & 63)) & 1ull;
}

struct Visit2 {
    uint64_t row;     // lane w: word w of corr64[ei]
    uint64_t z;       // lane w: word w of the OR of corr64[k], k in slot(ei), k != ei
    int x;            // lane t: popcount(corr64[ei] & B[t])
};

__device__ __forceinline__ void visit2_row_x(LsState& S, int ei, Visit2& V) {
    const int EW = S.EW, lane = S.lane;
    V.row = lane < EW ? S.pb.corr64[(size_t)ei * EW + lane] : 0ull;
    int x = 0;
    for (int w = 0; w < EW; ++w) {
        const uint64_t rw = readlane64(V.row, w);
        if (lane < kSlots) x += __popcll(rw & S.B[(size_t)lane * EW + w]);
    }
    V.x = x;
}

// the same from the visited event's row already in registers (lane w: word w)
__device__ __forceinline__ void visit2_x_from_row(LsState& S, uint64_t row, Visit2& V) {
    const int EW = S.EW, lane = S.lane;
    V.row = row;
    int x = 0;
    for (int w = 0; w < EW; ++w) {
        const uint64_t rw = readlane64(row, w);
        if (lane < kSlots) x += __popcll(rw & S.B[(size_t)lane * EW + w]);
    }
    V.x = x;
}

// corr64 row of event e, one word per lane (lanes < EW), for the next visit
__device__ __forceinline__ uint64_t load_row(const LsState& S, int e) {
    return S.lane < S.EW ? S.pb.corr64[(size_t)e * S.EW + S.lane] : 0ull;
}

__device__ __forceinline__ void visit2_z(LsState& S, int ei, Visit2& V) {
    const int EW = S.EW, lane = S.lane, ti = S.sl[ei];
    uint64_t z = 0;
    for (int w2 = 0; w2 < EW; ++w2) {
        const uint64_t bw = S.B[(size_t)ti * EW + w2];
        uint64_t m = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(bw >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)bw);
        if ((ei >> 6) == w2) m &= ~(1ull << (ei & 63));
        while (m) {
            const int k = 64 * w2 + __builtin_ctzll(m);
            m &= m - 1;
            if (lane < EW) z |= S.pb.corr64[(size_t)k * EW + lane];
        }
    }
    V.z = z;
}

// sum over words of popcount(row & set) for a row held one word per lane (lanes < EW)
__device__ __forceinline__ int row_in_set(const LsState& S, uint64_t row, const uint64_t* set) {
    return wave_sum(S.lane < S.EW ? __popcll(row & set[S.lane]) : 0);
}

// Slot s minus event `out` (-1: none) plus event `a` has a clash-free room
// matching (an augmenting path from `a` over the owner table).
__device__ __forceinline__ bool matchable(LsState& S, int s, int out, int a) {
    const int R = S.R, lane = S.lane;
    const int o = lane < R ? (int)S.hist[s * R + lane] : 0xFFFF;
    const bool valid = o != 0xFFFF && o != out;
    const uint64_t po = valid ? poss_of(S, o) : 0ull;
    const uint64_t used = ballot(valid);
    const uint64_t fre = (R >= 64 ? ~0ull : ((1ull << R) - 1)) & ~used;
    uint64_t seen = poss_of(S, a);
    if (seen & fre) return true;
    uint64_t fr = seen & used;
    while (fr) {
        const int r = __builtin_ctzll(fr);
        fr &= fr - 1;
        const uint64_t nx = readlane64(po, r) & ~seen;
        if (nx & fre) return true;
        seen |= nx;
        fr |= nx & used;
    }
    return false;
}

// ---- phase-1 room-pair lower bounds (TT_LS_P1B). A phase-1 trial from an
// infeasible state mostly fails on room clashes, which the correlation bounds
// above cannot see, so it used to run the full matcher of every touched slot
// just to be rejected. assignRooms (Solution.cpp:772-891) computes a MAXIMUM
// matching, so an unmatched event has no free possible room and goes to its
// first possible room, which is matched: each unmatched event with a possible
// room adds at least one clash pair. Hence for a touched slot s' (the current
// slot s, minus `out`, plus `a`):
//     pairs(s') >= |s'| - M(s') - Z(s')
// with Z the events without a possible room and M the maximum matching size;
// M(s + a) = M(s) + [augmenting path from a] exactly, and M(s - out + a) <=
// M(s + a) (a vertex removed never enlarges a matching). Per slot the kernel
// keeps a summary of one maximum matching: its matched rooms `used` and the
// rooms `fr` from which an alternating path (room -> its matched event -> a
// possible room of that event -> ...) reaches a free room, free rooms
// included. An augmenting path from a new event a exists iff poss(a) meets fr,
// so the bound costs a few bit operations per touched slot -- cheap enough
// for every lane of a trial window. The matching is read off the current
// rooms (a room holding an event for which it is possible has exactly one
// matched event; any such event will do) and checked: it is maximum iff no
// unmatched event has a possible room in fr (Berge); a slot that fails
// (rooms the caller chose, not assignRooms) is untrusted and gets no bound
// until an accepted move re-matches it with the reference matcher. A trial
// whose correlation bound plus these pair bounds already reaches the current
// value is rejected exactly as its full evaluation would reject it.
// The summaries are built out of line (plain arguments: a reference to LsState
// would put it in scratch): once per phase 1 and for a slot the lane-serial
// matcher re-matched, so their code stays out of the trial loops (the kernel's
// code grew 115 -> 136 KB with them inlined at every accept).
struct SinfView {
    SlotInfo* sinf;
    const uint64_t* B;
    const uint8_t* sl;
    const uint8_t* rr;
    const uint16_t* ps;
    const uint64_t* poss;
    uint8_t* task_base;
    int E, R, EW, scratch;
};
__device__ __forceinline__ SinfView sinf_view(const LsState& S) {
    return SinfView{S.sinf, S.B, S.sl, S.rr, S.ps, S.pb.poss, S.task_base, S.E, S.R, S.EW, S.scratch};
}
__device__ __forceinline__ uint64_t vposs(const SinfView& V, int e) { return V.ps ? (uint64_t)V.ps[e] : V.poss[e]; }
// The out-of-line summary functions get their view through LDS: sinf_init writes
// it into the wave's misc words [kSinfViewMisc, +12) -- LDS byte offsets of the
// arrays, the global possibleRooms pointer as two words, E, R, EW and the task
// scratch size -- and the functions take one pointer to it. (A SinfView passed
// by value is an aggregate in the caller's scratch frame, 72 B per lane; its
// fields as 19 argument registers measured +5..10 % on LS(200) from the call
// sites' register pressure, profiles/r06_ab_ls_scratch.jsonl.)
constexpr int kSinfViewMisc = 12;
extern __shared__ __attribute__((aligned(16))) uint8_t tt_ls_dyn[];   // the kernel's dynamic LDS
__device__ __forceinline__ void sinf_store_view(const LsState& S) {
    const int lane = S.lane;
    if (lane < 12) {
        const auto off = [](const void* q) { return q ? (int32_t)((const uint8_t*)q - tt_ls_dyn) : -1; };
        const uint64_t gp = (uint64_t)(uintptr_t)S.pb.poss;
        int32_t v = 0;
        switch (lane) {
            case 0: v = off(S.sinf); break;
            case 1: v = off(S.B); break;
            case 2: v = off(S.sl); break;
            case 3: v = off(S.rr); break;
            case 4: v = off(S.ps); break;
            case 5: v = off(S.task_base); break;
            case 6: v = (int32_t)(uint32_t)gp; break;
            case 7: v = (int32_t)(uint32_t)(gp >> 32); break;
            case 8: v = S.E; break;
            case 9: v = S.R; break;
            case 10: v = S.EW; break;
            default: v = S.scratch; break;
        }
        S.misc[kSinfViewMisc + lane] = v;
    }
    wave_sync();
}
__device__ __forceinline__ SinfView sinf_load_view(const int32_t* mv) {
    SinfView V;
    V.sinf = (SlotInfo*)(tt_ls_dyn + mv[0]);
    V.B = (const uint64_t*)(tt_ls_dyn + mv[1]);
    V.sl = tt_ls_dyn + mv[2];
    V.rr = tt_ls_dyn + mv[3];
    V.ps = mv[4] < 0 ? nullptr : (const uint16_t*)(tt_ls_dyn + mv[4]);
    V.task_base = tt_ls_dyn + mv[5];
    V.poss = (const uint64_t*)(uintptr_t)(((uint64_t)(uint32_t)mv[7] << 32) | (uint32_t)mv[6]);
    V.E = mv[8]; V.R = mv[9]; V.EW = mv[10]; V.scratch = mv[11];
    return V;
}
#define TT_SINF_PARAMS const int32_t *v_mv
#define TT_SINF_VIEW sinf_load_view(v_mv)
#define TT_SINF_ARGS(V) (V)

__device__ __noinline__ void sinf_build_v(TT_SINF_PARAMS, int t) {
    const SinfView V = TT_SINF_VIEW;
    const int R = V.R, EW = V.EW, lane = threadIdx.x & 63;
    uint16_t* own = (uint16_t*)V.task_base;               // scratch: free after accept's hist copies
    if (lane < R) own[lane] = 0xFFFF;
    wave_sync();
    for (int w = 0; w < EW; ++w) {
        const int e = 64 * w + lane;
        if ((V.B[(size_t)t * EW + w] >> lane) & 1ull) {
            const int r = V.rr[e];
            if ((vposs(V, e) >> r) & 1ull) own[r] = (uint16_t)e;
        }
    }
    wave_sync();
    const int o = lane < R ? (int)own[lane] : 0xFFFF;
    const bool valid = o != 0xFFFF;
    const uint64_t po = valid ? vposs(V, o) : 0ull;
    const uint64_t used = ballot(valid);
    uint64_t fr = (R >= 64 ? ~0ull : ((1ull << R) - 1)) & ~used;
    for (;;) {                                            // least fixed point, <= R rounds
        const uint64_t fn = fr | ballot(valid && (po & fr) != 0ull);
        if (fn == fr) break;
        fr = fn;
    }
    // N, Z and the maximality check (an unmatched event with a possible room in fr)
    int n = 0, z = 0;
    bool aug = false;
    for (int w = 0; w < EW; ++w) {
        const uint64_t bw = V.B[(size_t)t * EW + w];
        n += __popcll(bw);
        const int e = 64 * w + lane;
        const bool in = (bw >> lane) & 1ull;
        const uint64_t pe = in ? vposs(V, e) : 1ull;
        z += __popcll(ballot(pe == 0ull));
        if (in) aug |= own[V.rr[e]] != e && (pe & fr) != 0ull;
    }
    const bool trusted = !wave_any(aug);
    if (lane == 0) {
        V.sinf[t].used = (uint16_t)used;
        V.sinf[t].fr = (uint16_t)fr;
        V.sinf[t].nz = (trusted ? (int)0x80000000 : 0) | (n << 16) | z;
    }
    wave_sync();
}
__device__ __forceinline__ void sinf_build(LsState& S, int t) {
    sinf_build_v(S.misc + kSinfViewMisc, t);                  // the view sinf_init stored
}

// lower bound on the clash pairs of slot s minus `out` (-1: none) plus event a
// after the reference's re-match (0 for an untrusted slot); any lanes
__device__ __forceinline__ int pairs_lb_of(const SlotInfo& I, uint64_t pa, uint64_t pout, bool has_out) {
    const int nz = I.nz;
    if (nz >= 0) return 0;                                     // bit 31 clear: untrusted
    const int N = ((nz >> 16) & 0x7FFF) + (has_out ? 0 : 1);
    const int Z = (nz & 0xFFFF) + (pa == 0ull) - (has_out && pout == 0ull);
    const int u = N - __popc((uint32_t)I.used) - ((pa & (uint64_t)I.fr) != 0ull) - Z;
    return u > 0 ? u : 0;
}
__device__ __forceinline__ int pairs_lb(LsState& S, int s, int out, int a) {
    return pairs_lb_of(S.sinf[s], poss_of(S, a), out >= 0 ? poss_of(S, out) : 0ull, out >= 0);
}

// start of phase 1: the no-room event words and every slot's summary, all
// slots at once: owners of every (slot, room) in the matcher task scratch
// (free at this point), then the used masks, the fr fixed point over all
// slots together, and the maximality check (sinf_build slot by slot when
// the 45 x R owner table does not fit the task scratch)
__device__ __noinline__ void sinf_init_v(TT_SINF_PARAMS) {
    const SinfView V = TT_SINF_VIEW;
    const int E = V.E, R = V.R, lane = threadIdx.x & 63;
    const int NC = kSlots * R;
    if ((size_t)2 * NC > (size_t)V.scratch) {
        for (int t = 0; t < kSlots; ++t) sinf_build_v(v_mv, t);
        return;
    }
    uint16_t* own2 = (uint16_t*)V.task_base;                    // [45][R]
    const uint64_t rmask = R >= 64 ? ~0ull : ((1ull << R) - 1);
    const uint32_t rinv = ((1u << 20) + (uint32_t)R - 1) / (uint32_t)R;   // c / R = (c * rinv) >> 20 for c < 2^12
    for (int c = lane; c < NC; c += 64) own2[c] = 0xFFFF;
    if (lane < kSlots) { V.sinf[lane].used = 0; V.sinf[lane].fr = 0; V.sinf[lane].nz = (int)0x80000000; }
    wave_sync();
    for (int e = lane; e < E; e += 64) {
        const int t = V.sl[e], r = V.rr[e];
        const uint64_t pe = vposs(V, e);
        if ((pe >> r) & 1ull) own2[t * R + r] = (uint16_t)e;
        atomicAdd(&V.sinf[t].nz, (1 << 16) | (pe == 0ull ? 1 : 0));
    }
    wave_sync();
    for (int c = lane; c < NC; c += 64) {
        const int t = (int)(((uint32_t)c * rinv) >> 20), r = c - t * R;
        if (own2[c] != 0xFFFF) atomicOr((uint32_t*)&V.sinf[t], 1u << r);          // used: low half
    }
    wave_sync();
    if (lane < kSlots) V.sinf[lane].fr = (uint16_t)(rmask & ~(uint64_t)V.sinf[lane].used);
    wave_sync();
    for (;;) {                                                  // fr of every slot, least fixed point
        bool ch = false;
        for (int c = lane; c < NC; c += 64) {
            const int t = (int)(((uint32_t)c * rinv) >> 20), r = c - t * R;
            const int o = own2[c];
            const uint64_t f = V.sinf[t].fr;                   // (atomics below touch the high half only)
            if (o != 0xFFFF && !((f >> r) & 1ull) && (vposs(V, o) & f) != 0ull) {
                atomicOr((uint32_t*)&V.sinf[t], 1u << (16 + r));                     // fr: high half
                ch = true;
            }
        }
        wave_sync();
        if (!wave_any(ch)) break;
    }
    for (int e = lane; e < E; e += 64) {                        // Berge: no unmatched event reaches a free room
        const int t = V.sl[e];
        const uint64_t pe = vposs(V, e);
        if (pe != 0ull && own2[t * R + V.rr[e]] != e && (pe & (uint64_t)V.sinf[t].fr) != 0ull)
            atomicAnd(&V.sinf[t].nz, 0x7FFFFFFF);
    }
    wave_sync();
}
__device__ __forceinline__ void sinf_init(LsState& S) {
    LSP_T(t0);
    sinf_store_view(S);
    sinf_init_v(S.misc + kSinfViewMisc);
    LSP_ADD(S, kPfBInit, t0);
}

// ---- trial windows. A Move1/Move2 loop spends most of its trials on moves
// the cheap tests above reject. Up to 64 consecutive trials are screened at
// once, one per lane: lane k takes the trial k+1 draws ahead (Park-Miller jump:
// state * 16807^(k+1) mod (2^31 - 1), the exact value of k+1 Schrage steps),
// its draw, and whether it needs the full path; the step budget is applied
// as the scalar loop does (a trial runs only while step <= maxSteps, and only
// a passing draw costs a step). The first lane that needs the full path is
// run by the scalar code; the trials before it were rejected with their draws
// and steps consumed, exactly as one by one.
__device__ __forceinline__ int bperm(int v, int src_lane) { return __builtin_amdgcn_ds_bpermute(src_lane << 2, v); }
__device__ __forceinline__ uint64_t bperm64(uint64_t v, int src_lane) {
    return ((uint64_t)(uint32_t)bperm((int)(uint32_t)(v >> 32), src_lane) << 32) | (uint32_t)bperm((int)(uint32_t)v, src_lane);
}

// Resolves a window of `rem` remaining trials (lanes k < rem) whose per-lane
// full-path flag is `need`: returns the lane of the first trial to run in
// full (64: none), with st/step advanced past it (its draw and step taken);
// without one, past every trial the loop would have run, and done is set when
// the loop ends inside the window (step budget or its last trial).
__device__ __forceinline__ int window_resolve(int lane, uint32_t jump, int64_t& st, int& step, int max_steps, int rem,
                                              double p, bool need, bool& done) {
    const uint32_t sk = pm_mulmod((uint32_t)st, jump);
    const bool valid = lane < rem;
    const bool d = valid && __dmul_rn(1.0 / 2147483647.0, (double)sk) < p;
    const uint64_t dm = ballot(d);
    const uint64_t lt = (1ull << lane) - 1ull;
    const bool alive = valid && step + __popcll(dm & lt) <= max_steps;
    const uint64_t am = ballot(alive);
    const int kend = am == ~0ull ? 64 : __builtin_ctzll(~am);
    const uint64_t nm = ballot(alive && d && need);
    const int kstar = nm ? __builtin_ctzll(nm) : 64;
    const int last = kstar < 64 ? kstar : kend - 1;                    // last trial drawn
    if (last >= 0) {
        st = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)sk, last);
        step += __popcll(dm & (last == 63 ? ~0ull : ((2ull << last) - 1ull)));
    }
    done = kstar == 64 && (kend < 64 || rem <= 64);
    return kstar;
}

// x mod E for 0 <= x < E + 64 (scramble positions a window ahead): a subtraction
// or two instead of the integer division a runtime `% E` compiles to (dozens of
// scalar or vector instructions per use in the trial loops)
__device__ __forceinline__ int wrap_e(int x, int E) {
    while (x >= E) x -= E;
    return x;
}

// TT_LS_HOT (phase 1): the events with eventHcv > 0 as a bitmask over event
// ids, one word per lane (lane w: events 64w..64w+63). A visit of an event
// with eventHcv == 0 only counts towards evCount (no draw, no step:
// Solution.cpp:509-512), so the visit loop jumps over such events 64 scramble
// positions at a time instead of loading each one's correlation row. The flags
// change only for the events of the slots an accepted move touches
// (eventHcv(e) depends on e's slot only), which refresh_hot recomputes. Used
// when at most a quarter of the events have eventHcv > 0 at the start of phase 1
// (a GA child of feasible parents); from a random solution nearly every event
// is visited anyway and the flags' upkeep after every accepted move only costs.
// (The flags in LDS instead of a register measured slower: 136 VGPRs spilled.)
#ifndef TT_LS_HOT
#define TT_LS_HOT 1
#endif
// The flags of events 64k + lane; with `all` every event, else
// only those in a touched slot (S.ts, after accept) replace their flag in `hot`
// (lane k holds word k)
__device__ __forceinline__ uint64_t refresh_hot(LsState& S, uint64_t hot, bool all) {
    LSP_T(t0);
    const int E = S.E, R = S.R, EW = S.EW, lane = S.lane;
    for (int k = 0; 64 * k < E; ++k) {                        // wave-uniform
        const int e = 64 * k + lane;
        bool upd = false, h = false;
        if (e < E) {
            const int t = S.sl[e];
            upd = all || (S.nts > 0 && t == S.ts[0]) || (S.nts > 1 && t == S.ts[1]) || (S.nts > 2 && t == S.ts[2]);
            if (upd) {
                const int c = (int)S.hist[t * R + S.rr[e]] - 1 +
                              row_pop_in(S.pb.corr64 + (size_t)e * EW, S.B + (size_t)t * EW, EW, e);
                h = c > 0;
            }
        }
        const uint64_t um = ballot(upd), hm = ballot(h);
        if (um && lane == k) hot = (hot & ~um) | hm;
    }
    LSP_ADD(S, kPfHot1, t0);
    return hot;
}

// One individual's localSearch by the calling wave (every lane). CAP =
// matcher task capacity. redo_list (first launch, CAP = kLsCapSmall): an
// individual that overflowed a task is appended to it (redo_list[0] counts,
// entries from redo_list[2], at most redo_cap of them: beyond that status bit
// 4 is set) and its HBM row and stream are left as they were; NULL when no
// task can overflow.
// Optional evaluation of the searched individual (tt_local_search_eval): the
// localSearch -> computePenalty pair of ga.cpp:574-575 in one launch, so a GA
// generation needs no separate evaluation of its children after the search.
struct LsEvalOut {
    int32_t* hcv;
    int32_t* scv;
    uint8_t* feasible;
    int32_t* penalty;
};

// computeFeasibility / computeHcv / computeScv / computePenalty
// (Solution.cpp:63-170) of the individual in the wave's LDS state (slots sl,
// rooms rr, slot bitsets B), in tt_eval.hip's closed forms:
//   hcv = sum over (slot, room) cells of C(n, 2)          (:148-150)
//       + #{i < j : same slot, correlated}                  (:151-153)
//       + #{e : room not possible for e}                    (:155-156)
//   scv = sum_e [slot_e % 9 == 8] studentNumber(e)          (:93-96)
//       + sum over students of the >2-in-a-row and single-class terms of the
//         student's slot mask                               (:99-137)
// The room histogram is rebuilt from the rows (phase 2 keeps an owner table there).
__device__ __forceinline__ void ls_eval(LsState& S, long p, const LsEvalOut& out) {
    const DevProblem& pb = S.pb;
    const int E = S.E, R = S.R, EW = S.EW, lane = S.lane;
    for (int c = lane; c < kSlots * R; c += 64) S.hist[c] = 0;
    wave_sync();
    int h = 0, sc = 0;
    if (lane < kSlots) {                                   // room clash pairs of slot `lane`
        for (int w = 0; w < EW; ++w) {
            uint64_t x = S.B[(size_t)lane * EW + w];
            while (x) {
                const int e = 64 * w + __builtin_ctzll(x);
                x &= x - 1;
                const int r = S.rr[e];
                h += S.hist[lane * R + r];
                S.hist[lane * R + r] = (uint16_t)(S.hist[lane * R + r] + 1);
            }
        }
    }
    int cp = 0;                                            // 2 x correlated pairs
    for (int e = lane; e < E; e += 64) {
        const int t = S.sl[e], r = S.rr[e];
        cp += row_pop_in(pb.corr64 + (size_t)e * EW, S.B + (size_t)t * EW, EW, e);   // minus corr(e, e): e has a student
        h += (int)(((pb.poss[e] >> r) & 1ull) ^ 1ull);
        if ((kLastSlotMask >> t) & 1ull) sc += pb.sn[e];
    }
    for (int st = lane; st < pb.S; st += 64) {
        uint64_t m = 0;
        for (int k = pb.stu_off[st]; k < pb.stu_off[st + 1]; ++k) m |= 1ull << S.sl[pb.stu_ev[k]];
        sc += mask_scv(m);
    }
    h = wave_sum(h);
    cp = wave_sum(cp);
    sc = wave_sum(sc);
    if (lane == 0) {
        const int hcv = h + cp / 2;
        out.hcv[p] = hcv;
        out.scv[p] = sc;
        out.feasible[p] = hcv == 0 ? 1 : 0;
        out.penalty[p] = hcv == 0 ? sc : 1000000 + hcv;
    }
}

template <int CAP>
__device__ __attribute__((always_inline)) inline void ls_one(const DevProblem& pb, uint8_t* __restrict__ slot,
                                                             uint8_t* __restrict__ room, int64_t* __restrict__ rng,
                                                             long p, int max_steps, double p1, double p2, double p3,
                                                             int32_t* __restrict__ redo_list, int redo_cap, int smS,
                                                             unsigned long long* __restrict__ ph_steps,
                                                             const LsEvalOut& eout) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int E = pb.E, R = pb.R, EW = pb.EW64;
    const int lane = threadIdx.x;
    LSP_T(t_kernel);
#ifdef TT_LS_PROF
    const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef TT_LS_PROF
    uint64_t t_ph = 0;                  // phase timer (assigned, not declared, between the gotos and redo:)
#endif
    const LsLayout L = ls_layout(E, R, EW, CAP, smS);
    LsState S;
    S.pb = pb; S.E = E; S.R = R; S.EW = EW; S.lane = lane;
    S.sl = lds + L.sl; S.rr = lds + L.rr; S.nrr = lds + L.nrr;
    S.evl = (uint16_t*)(lds + L.evl);
    S.pos = (uint16_t*)(lds + L.pos); S.slp = lds + L.slp;
    S.B = (uint64_t*)(lds + L.B); S.NB = (uint64_t*)(lds + L.NB);
    S.ps = (TT_LS_POSS16 && R <= 16) ? (const uint16_t*)(lds + L.ps) : nullptr;
    S.sm = nullptr;
    S.rp = (int32_t*)(lds + L.rp); S.hist = (uint16_t*)(lds + L.hist);
    S.misc = (int32_t*)(lds + L.misc);
    S.task_base = lds + L.task;
    S.task_bytes = (int)L.task_bytes;
    S.scratch = (int)L.scratch;
    S.NT = L.NT;
    S.nmv = 0; S.nts = 0;
    S.c1_valid = 0;
    S.listed = 0;
    S.phase2 = 0;
    S.sinf = nullptr; S.tvalid = 0;
#ifdef TT_LS_PROF
#pragma unroll
    for (int i = 0; i < kPfN; ++i) S.prof[i] = 0;
#endif
    if (lane == 0) S.misc[3] = 0;
    const uint32_t jump = pm_pow(lane + 1);                             // lane k: k+1 draws ahead

    // ---- load the individual, derive the incremental state
    bool bad = false;
    for (int e = lane; e < E; e += 64) {
        const uint8_t s = slot[p * E + e], r = room[p * E + e];
        bad |= s >= kSlots || r >= R;
        S.sl[e] = s; S.rr[e] = r; S.nrr[e] = r; S.evl[e] = (uint16_t)e;
    }
    if (lane == 0) S.sl[E] = 63;
    if (S.ps)
        for (int e = lane; e < E; e += 64) ((uint16_t*)S.ps)[e] = (uint16_t)pb.poss[e];
    for (int c = lane; c < kSlots * EW; c += 64) S.B[c] = 0ull;
    for (int c = lane; c < kSlots * R; c += 64) S.hist[c] = 0;
    __syncthreads();
    if (wave_any(bad)) {                       // invalid genome: leave it untouched
        if (lane == 0) {
            atomicOr(pb.status, 2);
            if (eout.hcv) {                    // tt_eval's sentinels for an invalid genome
                eout.hcv[p] = -1; eout.scv[p] = -1; eout.feasible[p] = 0; eout.penalty[p] = -1;
            }
        }
        return;
    }
    for (int e = lane; e < E; e += 64) {
        const int s = S.sl[e];
        atomicOr((unsigned long long*)&S.B[(size_t)s * EW + (e >> 6)], 1ull << (e & 63));
    }
    __syncthreads();
    if (lane < kSlots) {                    // room histogram + clash pairs of every slot
        int pairs = 0;
        for (int w = 0; w < EW; ++w) {
            uint64_t x = S.B[(size_t)lane * EW + w];
            while (x) {
                const int e = 64 * w + __builtin_ctzll(x);
                x &= x - 1;
                const int r = S.rr[e];
                pairs += S.hist[lane * R + r];
                S.hist[lane * R + r] = (uint16_t)(S.hist[lane * R + r] + 1);
            }
        }
        S.rp[lane] = pairs;
    }
    __syncthreads();

    LSP_T(t_scr);
    int64_t st = rng[p];
    // scramble the event list (Solution.cpp:476-484): swap i with a draw j_i for
    // i = 0..E-1. The draws do not depend on the list, so they are taken 64 at a
    // time, one per lane (lane k: state * 16807^(k+1), the Park-Miller jump; the
    // first draws by Schrage, until an out-of-range seed is brought into range), and
    // lane 0 then applies the block's swaps in order: only the LDS round trips of
    // the swaps stay serial.
    {
        int i = 0;
        // Schrage steps until the state is in range (one step, except for seeds >= 2^31)
        for (; i < E && (i == 0 || (uint64_t)st >= kPmM); ++i) {
            const int j = pm_pick(st, E);
            if (lane == 0) {
                const uint16_t h = S.evl[i];
                S.evl[i] = S.evl[j];
                S.evl[j] = h;
            }
        }
        for (int i0 = i; i0 < E; i0 += 64) {
            const int n = min(64, E - i0);
            const uint32_t sk = pm_mulmod((uint32_t)st, jump);
            const int jk = (int)__dmul_rn(__dmul_rn(1.0 / 2147483647.0, (double)sk), (double)E);
            st = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)sk, n - 1);
            for (int k = 0; k < n; ++k) {
                const int j = __builtin_amdgcn_readlane(jk, k);
                if (lane == 0) {
                    const uint16_t h = S.evl[i0 + k];
                    S.evl[i0 + k] = S.evl[j];
                    S.evl[j] = h;
                }
            }
        }
    }
    __syncthreads();
#if TT_LS_SLP
    for (int q = lane; q < E; q += 64) {
        const int e = S.evl[q];
        S.pos[e] = (uint16_t)q;
        S.slp[q] = S.sl[e];
    }
    __syncthreads();
#endif
    LSP_ADD(S, kPfScramble, t_scr);

    LSP_ADD(S, kPfInit, t_kernel);
    int step = 0, evc = 0;
    bool better = false;
    // Defensive bound on event visits, never reached: every visit either counts
    // towards evc < E or accepts a trial (which costs a step and resets evc), so a
    // phase makes at most (max_steps + 2) * E visits (Solution.cpp:498-505,616-618)
    // and both phases together at most half of guard_max. Status bit 2 reports it;
    // tests/test_gpu_parity.py asserts it never fires.
    const long guard_max = 4l * (long)E * ((long)max_steps + 2) + 1024;
    long guard = 0;
    const bool fast1 = EW <= 64;                                        // row words fit the lanes
    LSP_SET(t_ph);
    if (!feasible_now(S)) {                                             // phase 1 (Solution.cpp:497-618)
        // TT_LS_ROWPF: the visited event's correlation row loaded one visit ahead
        // (the scrambled event list is fixed, so the next visit's event is known)
        uint64_t nrow = (fast1 && TT_LS_ROWPF) ? load_row(S, S.evl[0]) : 0ull;
        uint64_t hot = 0;
        int nhot = 0;
        if (TT_LS_HOT && fast1) {
            hot = refresh_hot(S, 0ull, true);
            nhot = wave_sum(lane < EW ? __popcll(hot) : 0);
        }
        const bool hotm = TT_LS_HOT && fast1 && 4 * nhot <= E;
        // many events in conflict: room-pair lower bounds before the matcher (TT_LS_P1B)
#ifndef TT_LS_P1B_RTOFF
#define TT_LS_P1B_RTOFF 0       // profiling: the bounds compiled in but never enabled (p1 < 2 always)
#endif
        if (TT_LS_P1B && R <= kP1bMaxRooms && !hotm && fast1 && !(TT_LS_P1B_RTOFF && p1 < 2.0)) {
            S.sinf = (SlotInfo*)(lds + L.sinf);
            sinf_init(S);
        }
        if (S.sinf) {
#define TT_P1 1
#include "tt_ls_phase1.inc"
#undef TT_P1
        } else {
            S.sinf = nullptr;                    // known null in this copy (accept, matcher)
#define TT_P1 0
#include "tt_ls_phase1.inc"
#undef TT_P1
        }
    }
    LSP_ADD(S, kPfPh1, t_ph);
    LSP_SET(t_ph);
    if (feasible_now(S)) {                                              // phase 2 (Solution.cpp:619-768)
        // owner table in place of the room histogram (rooms are distinct per slot now)
        S.phase2 = 1;
        S.sinf = nullptr;
        if (ph_steps && lane == 0) S.misc[8] = step;                   // phase-1 steps (for the statistics)
        for (int c = lane; c < kSlots * R; c += 64) S.hist[c] = 0xFFFF;
        if (TT_LS_SMASK && smS > 0) {
            S.sm = (uint64_t*)(lds + L.sm);
            for (int st = lane; st < pb.S; st += 64) {
                uint64_t m = 0;
                for (int c = pb.stc_off[st]; c < pb.stc_off[st + 1]; ++c) m |= 1ull << (S.sl[pb.stc_ev[c]] & 63);
                S.sm[st] = m;
            }
        }
        wave_sync();
        for (int e = lane; e < E; e += 64) S.hist[S.sl[e] * R + S.rr[e]] = (uint16_t)e;
        wave_sync();
        const bool fast = fast1;
        evc = 0;
        uint64_t nrow = (fast && TT_LS_ROWPF) ? load_row(S, S.evl[0]) : 0ull;
        for (int i = 0; evc < E; i = wrap_e(i + 1, E)) {
            if (step > max_steps || ++guard > guard_max) break;
            const int ei = S.evl[i];
            LSP_CNT(S, kPfVisits);
            LSP_T(t_vis);
            uint64_t row = nrow;
            if (fast && TT_LS_ROWPF) nrow = load_row(S, S.evl[i + 1 < E ? i + 1 : 0]);
            else if (fast) row = load_row(S, ei);
            int cur, scs_i;
            scv_terms(S, ei, false, cur, scs_i);
            if (cur == 0) { evc++; LSP_ADD(S, kPfVis2, t_vis); continue; }
            const int ti = S.sl[ei];
            Visit2 V;
            if (fast) visit2_x_from_row(S, row, V);
            LSP_ADD(S, kPfVis2, t_vis);
            LSP_T(t_m1);
            const int t_start = pm_pick(st, kSlots);
            for (int h = 0; h < kSlots;) {
                if (step > max_steps) break;
                const bool win = fast && (uint64_t)st < kPmM;
                if (win) {
                    // window: lane k screens target t_start+h+k (ei must meet no correlated event there)
                    const int rem = kSlots - h;
                    const int tk = (t_start + h + lane) % kSlots;
                    const int xt = bperm(V.x, tk);                          // every lane takes part
                    const bool need = lane < rem && (tk == ti || xt == 0);
                    bool done;
                    const int ks = window_resolve(lane, jump, st, step, max_steps, rem, p1, need, done);
                    if (ks == 64) break;                                // rem <= 45 < 64: the loop ends here
                    h += ks;
                } else {
                    if (!(pm_next(st) < p1)) { h++; continue; }
                    step++;
                }
                const int t = (t_start + h) % kSlots;
                h++;
                if (fast && t != ti) {
                    // ei meets a correlated event in t, or t cannot take ei without a clash
                    LSP_CNT(S, kPfQ1);
                    if (__builtin_amdgcn_readlane(V.x, t) != 0) continue;
                    LSP_CNT(S, kPfQ1c);
                    if (!matchable(S, t, -1, ei)) continue;
                    LSP_CNT(S, kPfQ1m);
                }
                set_move(S, 1, ei, t, 0);
                build_nb(S);
                // eah_nb(ei) == 0 needs no correlated event in t (no rooms needed)
                // and no room clash in t (task 0); the old slot (task 1) is
                // matched only for an accepted move
                if (!(fast && t != ti) && corr_nb(S, ei) != 0) continue;
                if (match_tasks(S, 1)) goto redo;
                if (S.misc[0] == 0) {
                    int es_n, scs_n;
                    scv_terms(S, ei, true, es_n, scs_n);
                    if (es_n + scs_i - scs_n < cur) {
                        if (match_tasks(S, 2)) goto redo;
                        accept(S); evc = 0; better = true; break;
                    }
                }
                restore_task<0>(S);
            }
            cache_drop(S);
            LSP_ADD(S, kPfM1p2, t_m1);
            if (better) { better = false; continue; }
            if (p2 != 0) {
                LSP_T(t_m2);
                if (fast) visit2_z(S, ei, V);
                int j = wrap_e(i + 1, E);
                while (j != i) {
                    if (step > max_steps) break;
                    if (fast && (uint64_t)st < kPmM) {
                        // window: lane k screens partner j+k (no correlated event for either
                        // moved event in its new slot)
                        const int rem = wrap_e(i - j + E, E);
                        // (ds_bpermute reads 0 from inactive lanes: every lane takes part)
#if TT_LS_SLP
                        int pk = j + lane;
                        if (pk >= E) pk -= E;
                        if (pk >= E) pk %= E;                      // E < 64 only
                        const int ej = S.evl[pk], tj = S.slp[pk];
#else
                        const int ej = S.evl[wrap_e(j + lane, E)], tj = S.sl[ej];
#endif
                        const uint64_t rw = bperm64(V.row, ej >> 6), zw = bperm64(V.z, ej >> 6);
                        const int xt = bperm(V.x, tj);
                        bool need = true;
                        if (lane < rem && tj != ti) {
                            const int cij = (int)((rw >> (ej & 63)) & 1ull);
                            need = xt - cij == 0 && !((zw >> (ej & 63)) & 1ull);
                        }
                        bool done;
                        const int ks = window_resolve(lane, jump, st, step, max_steps, rem, p2, need, done);
                        if (ks == 64) {
                            if (done) break;
                            j = wrap_e(j + 64, E);
                            continue;
                        }
                        j = wrap_e(j + ks, E);
                    } else {
                        if (!(pm_next(st) < p2)) { j = wrap_e(j + 1, E); continue; }
                        step++;
                    }
                    // ---- the full trial at j (its draw and step taken)
                    bool acc = false;
                    do {
                        const int ej = S.evl[j];
                        const int tj = S.sl[ej];
                        const bool quick = fast && tj != ti;
                        if (quick) {
                            // corr_nb(ei) = X[tj] - corr(ei, ej); corr_nb(ej) = 0 iff no slot-mate of ei
                            // is correlated with ej; then both slots must match without a clash
                            LSP_CNT(S, kPfQ2);
                            if (__builtin_amdgcn_readlane(V.x, tj) - (int)row_bit(V.row, ej) != 0) break;
                            if (row_bit(V.z, ej)) break;
                            LSP_CNT(S, kPfQ2c);
                            if (!matchable(S, tj, ej, ei) || !matchable(S, ti, ei, ej)) break;
                            LSP_CNT(S, kPfQ2m);
                        }
                        set_move(S, 2, ei, ej, 0);
                        build_nb(S);
                        if (!quick && corr_nb(S, ei) + corr_nb(S, ej) != 0) break;   // eah_nb > 0 whatever the rooms
                        const TaskRegs tr = load_tasks(S, 7);
                        if (S.nts == 2) {
                            if (match_tasks(S, 1, tr)) goto redo;
                            if (S.misc[0] != 0) { restore_task<0>(S); break; }
                            if (match_tasks(S, 2, tr)) goto redo;
                        } else if (match_tasks(S, 7, tr)) goto redo;
                        if (S.misc[task_of(S, slot_nb(S, ei))] + S.misc[task_of(S, slot_nb(S, ej))] == 0) {
                            int es_ni, scs_ni, es_nj, scs_nj, es_cj, scs_cj;
                            scv_terms(S, ei, true, es_ni, scs_ni);
                            scv_terms(S, ej, true, es_nj, scs_nj);
                            scv_terms(S, ej, false, es_cj, scs_cj);
                            const int n = es_ni + scs_i - scs_ni + es_nj + scs_cj - scs_nj;
                            if (n < cur + es_cj) { accept(S); acc = true; break; }
                        }
                        sync_rooms(S, false);
                    } while (0);
                    if (acc) { evc = 0; better = true; break; }
                    j = wrap_e(j + 1, E);
                }
                LSP_ADD(S, kPfM2p2, t_m2);
                if (better) { better = false; continue; }
            }
            if (p3 != 0) {
                for (int j = wrap_e(i + 1, E); j != i; j = wrap_e(j + 1, E)) {
                    if (step > max_steps) break;
                    for (int k = wrap_e(j + 1, E); k != i; k = wrap_e(k + 1, E)) {
                        if (step > max_steps) break;
                        const int ej = S.evl[j], ek = S.evl[k];
                        for (int order = 0; order < 2; ++order) {
                            if (order == 1 && step > max_steps) break;
                            if (!(pm_next(st) < p3)) continue;
                            step++;
                            const int a = order ? ek : ej, b = order ? ej : ek;
                            set_move(S, 3, ei, a, b);
                            if (build_and_match(S)) goto redo;
                            if (eah_nb(S, ei) + eah_nb(S, a) + eah_nb(S, b) == 0) {
                                int es_ni, scs_ni, es_na, scs_na, es_nb, scs_nb, es_ca, scs_ca, es_cb, scs_cb;
                                scv_terms(S, ei, true, es_ni, scs_ni);
                                scv_terms(S, a, true, es_na, scs_na);
                                scv_terms(S, b, true, es_nb, scs_nb);
                                scv_terms(S, a, false, es_ca, scs_ca);
                                scv_terms(S, b, false, es_cb, scs_cb);
                                const int n = es_ni + scs_i - scs_ni + es_na + scs_ca - scs_na + es_nb + scs_cb - scs_nb;
                                if (n < cur + es_ca + es_cb) { accept(S); evc = 0; better = true; break; }
                            }
                            sync_rooms(S, false);
                        }
                        if (better) break;
                    }
                    if (better) break;
                }
                if (better) { better = false; continue; }
            }
            evc++;
        }
    }
    LSP_ADD(S, kPfPh2, t_ph);
    if (guard > guard_max && lane == 0) atomicOr(pb.status, 4);
    if (ph_steps && lane == 0) {                 // phase-2 steps, all steps (vector atomics, one lane)
        atomicAdd(&ph_steps[0], (unsigned long long)(S.phase2 ? step - S.misc[8] : 0));
        atomicAdd(&ph_steps[1], (unsigned long long)step);
    }

    __syncthreads();
    for (int e = lane; e < E; e += 64) {
        slot[p * E + e] = S.sl[e];
        room[p * E + e] = S.rr[e];
    }
    if (lane == 0) rng[p] = st;
    if (eout.hcv) ls_eval(S, p, eout);
#ifdef TT_LS_PROF
    LSP_ADD(S, kPfTotal, t_kernel);
    LSP_CNT(S, kPfWaves);
    if (lane == 0 && p < kLsWaveRec) {
        g_ls_wave[4 * p] = rt_start;
        g_ls_wave[4 * p + 1] = __builtin_amdgcn_s_memrealtime();
        g_ls_wave[4 * p + 2] = S.prof[kPfTotal];
        g_ls_wave[4 * p + 3] = S.prof[kPfTrials];
    }
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < kPfN; ++i)
            if (i != kPfMaxTotal) atomicAdd(&g_ls_prof[i], (unsigned long long)S.prof[i]);
        atomicMax(&g_ls_prof[kPfMaxTotal], (unsigned long long)S.prof[kPfTotal]);   // the slowest wave
    }
#endif
    return;
redo:
    if (lane == 0) {
        const int k = atomicAdd(&redo_list[0], 1);
        if (k < redo_cap) redo_list[2 + k] = (int32_t)p;
        else atomicOr(pb.status, 16);
    }
}

#ifndef TT_LS_WPE
#define TT_LS_WPE 5
#endif
// First launch: one wave per individual, in dispatch order `order` (NULL:
// 0..P-1; entries outside 0..P-1 are skipped, tt_local_search_ordered checks
// the permutation).
template <int CAP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(TT_LS_WPE))) void local_search_kernel(
    DevProblem pb, uint8_t* __restrict__ slot, uint8_t* __restrict__ room, int64_t* __restrict__ rng, int P,
    int max_steps, double p1, double p2, double p3, int32_t* __restrict__ redo_list, int redo_cap,
    const int32_t* __restrict__ order, int smS, unsigned long long* __restrict__ ph_steps, LsEvalOut eout) {
    const long p = order ? (long)order[blockIdx.x] : (long)blockIdx.x;   // dispatch order only
    if ((unsigned long)p >= (unsigned long)P) return;
    ls_one<CAP>(pb, slot, room, rng, p, max_steps, p1, p2, p3, redo_list, redo_cap, smS, ph_steps, eout);
}

// Redo launch: a grid of resident waves works through the individuals the
// first launch listed, with full-size matcher tasks; the last wave to finish
// resets the list for the stream's next call (no per-call memset). With an
// empty list every wave returns at once (the arrival count is only needed when
// there is a list to reset: 52 -> a few us per GA generation).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(TT_LS_WPE))) void local_search_redo_kernel(
    DevProblem pb, uint8_t* __restrict__ slot, uint8_t* __restrict__ room, int64_t* __restrict__ rng, int max_steps,
    double p1, double p2, double p3, int32_t* __restrict__ redo_list, int redo_cap, int smS,
    unsigned long long* __restrict__ ph_steps, LsEvalOut eout) {
    const int n = min(redo_list[0], redo_cap);
    if (n == 0) return;             // nothing listed: every wave sees 0, no reset needed (no arrival atomics)
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        __syncthreads();
        ls_one<kMaxSlotEvents>(pb, slot, room, rng, (long)redo_list[2 + i], max_steps, p1, p2, p3, nullptr, 0, smS,
                               ph_steps, eout);
    }
    __threadfence();
    if (threadIdx.x == 0 && atomicAdd(&redo_list[1], 1) == (int)gridDim.x - 1) {
        redo_list[0] = 0;                                   // every wave has read the count
        redo_list[1] = 0;
    }
}

// Permutation check of a dispatch order (status bit 3 when it is not one),
// exact: every entry in 0..P-1 and none seen twice (P entries in range with no
// duplicate are a permutation). One workgroup marks the entries in a visited
// bitmap in LDS, `bits` entries per pass (every pass reads the whole order).
__global__ __launch_bounds__(1024) void order_check_kernel(const int32_t* __restrict__ order, int P, int bits,
                                                           int32_t* __restrict__ status) {
    extern __shared__ uint32_t seen[];
    __shared__ int bad_any;
    if (threadIdx.x == 0) bad_any = 0;
    bool bad = false;
    for (int lo = 0; lo < P; lo += bits) {
        const int hi = min(P, lo + bits);
        for (int w = threadIdx.x; w < (hi - lo + 31) / 32; w += 1024) seen[w] = 0u;
        __syncthreads();
        for (int i = threadIdx.x; i < P; i += 1024) {
            const int v = order[i];
            if (lo == 0) bad |= v < 0 || v >= P;
            if (v >= lo && v < hi) {
                const uint32_t bit = 1u << ((v - lo) & 31);
                bad |= (atomicOr(&seen[(v - lo) >> 5], bit) & bit) != 0u;
            }
        }
        __syncthreads();
    }
    if (bad) atomicOr(&bad_any, 1);
    __syncthreads();
    if (threadIdx.x == 0 && bad_any) atomicOr(status, 8);
}

}  // namespace ttga

using namespace ttga;

#ifdef TT_LS_PROF
extern "C" int tt_ls_wave_read(unsigned long long* out, int reset) {
    TT_HIP(hipDeviceSynchronize());
    TT_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ls_wave), sizeof(unsigned long long) * 4 * kLsWaveRec));
    if (reset) {
        std::vector<unsigned long long> z(4 * kLsWaveRec, 0ull);
        TT_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_ls_wave), z.data(), sizeof(unsigned long long) * 4 * kLsWaveRec));
    }
    return kLsWaveRec;
}
extern "C" int tt_ls_prof_read(unsigned long long* out, int reset) {
    TT_HIP(hipDeviceSynchronize());
    TT_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ls_prof), sizeof(unsigned long long) * kPfN));
    if (reset) {
        unsigned long long z[kPfN] = {};
        TT_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_ls_prof), z, sizeof(z)));
    }
    return kPfN;
}
#endif

// Phase-2 masks for kernel k at cap: the workgroups per CU without and with
// them, (o0 << 8) | o1 (0: no masks for this instance)
template <typename K>
static int ls_mask_occupancy(const tt_problem* p, int cap, K k) {
    const int S = p->dev.S;
    if (!TT_LS_SMASK || S <= 0 || 8 * (size_t)S > kSmaskMaxBytes) return 0;
    const size_t b0 = ls_layout(p->E, p->R, p->dev.EW64, cap, 0).bytes, b1 = ls_layout(p->E, p->R, p->dev.EW64, cap, S).bytes;
    int o0 = 0, o1 = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o0, k, 64, b0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&o1, k, 64, b1) != hipSuccess || o1 < 1) {
        (void)hipGetLastError();
        return 0;
    }
    o0 = std::min(o0, lds_resident_limit(b0));
    o1 = std::min(o1, lds_resident_limit(b1));
    if (o1 < 1) return 0;
    return (std::min(o0, 255) << 8) | std::min(o1, 255);
}

// students with phase-2 masks for a launch of P waves: S where the masks cost no
// resident waves -- the same occupancy with them, or P small enough that every
// CU holds all its waves at once with them -- or where they cost waves but an
// earlier call on the stream spent at least kLsMaskShare of its steps in phase 2
// (phase2 / all, -1: unknown); else 0. Measured on the GA at 8,192 children
// (profiles/r05_ab_ga_ls_masks.jsonl): masks at 18 instead of 20 waves per CU
// give comp01 (mostly phase 2) +5 %, comp10 -2 % and comp15 (phase 1 only) -4 %.
// The masks never change a result, only the launch's speed.
constexpr double kLsMaskShare = TT_LS_MASK_SHARE;
template <typename K>
static int ls_mask_students(const tt_problem* p, int cap, K k, int P, double share2 = -1.0) {
    std::atomic<int>& memo = const_cast<tt_problem*>(p)->ls_smask[cap == kMaxSlotEvents ? 0 : 1];
    int m = memo.load(std::memory_order_relaxed);
    if (m < 0) memo.store(m = ls_mask_occupancy(p, cap, k), std::memory_order_relaxed);
    if (m == 0) return 0;
#ifdef TT_LS_SMASK_FORCE
    return p->dev.S;                            // profiling: masks whatever the occupancy
#endif
    const int o0 = m >> 8, o1 = m & 255;
    const long per_cu = ((long)P + p->num_cus - 1) / p->num_cus;
    return (o1 >= o0 || per_cu <= o1 || share2 >= kLsMaskShare) ? p->dev.S : 0;
}

// entries of a dispatch order checked per pass of order_check_kernel (128 KB of LDS)
constexpr int kOrderCheckBits = 128 * 1024 * 8;

// the stream's redo record (ls_mu held)
static tt_problem::LsRedo* find_redo(tt_problem* mp, void* stream) {
    for (auto& r : mp->ls_redo)
        if (r.stream == stream) return &r;
    return nullptr;
}

extern "C" int tt_local_search_stats(const tt_problem* p, void* stream, uint64_t* steps) {
    if (!p || !steps) { set_error("null argument"); return TT_ERR_INVALID; }
    tt_problem* mp = const_cast<tt_problem*>(p);
    steps[0] = steps[1] = 0ull;
    hipEvent_t ev = nullptr;
    int slot = 0;
    {
        std::lock_guard<std::mutex> lock(mp->ls_mu);
        const tt_problem::LsRedo* r = find_redo(mp, stream);
        if (!r || r->calls == 0) return TT_OK;
        slot = (int)((r->calls - 1) & 1);
        ev = r->ev[slot];
    }
    const int rc = use_device(p);
    if (rc) return rc;
    if (ev) TT_HIP(hipEventSynchronize(ev));        // the last call's counts have landed
    std::lock_guard<std::mutex> lock(mp->ls_mu);
    const tt_problem::LsRedo* r = find_redo(mp, stream);
    if (r && r->ph_host) {
        steps[0] = r->ph_host[2 * slot];
        steps[1] = r->ph_host[2 * slot + 1];
    }
    return TT_OK;
}

extern "C" int tt_local_search_masks(const tt_problem* p, void* stream, int32_t* students) {
    if (!p || !students) { set_error("null argument"); return TT_ERR_INVALID; }
    tt_problem* mp = const_cast<tt_problem*>(p);
    std::lock_guard<std::mutex> lock(mp->ls_mu);
    const tt_problem::LsRedo* r = find_redo(mp, stream);
    *students = r && r->calls > 0 ? r->sms_last : -1;
    return TT_OK;
}

extern "C" int tt_local_search(const tt_problem* p, uint8_t* slot, uint8_t* room, int64_t* rng, int P,
                               int max_steps, double p1, double p2, double p3, void* stream) {
    return tt_local_search_ordered(p, slot, room, rng, P, max_steps, p1, p2, p3, nullptr, stream);
}

extern "C" int tt_local_search_ordered(const tt_problem* p, uint8_t* slot, uint8_t* room, int64_t* rng, int P,
                                       int max_steps, double p1, double p2, double p3, const int32_t* order,
                                       void* stream) {
    return tt_local_search_eval(p, slot, room, rng, P, max_steps, p1, p2, p3, order, nullptr, nullptr, nullptr,
                                nullptr, stream);
}

extern "C" int tt_local_search_eval(const tt_problem* p, uint8_t* slot, uint8_t* room, int64_t* rng, int P,
                                    int max_steps, double p1, double p2, double p3, const int32_t* order,
                                    int32_t* hcv, int32_t* scv, uint8_t* feasible, int32_t* penalty, void* stream) {
    int rc = check_pop_args(p, P, slot, room);
    if (rc || P == 0) return rc;
    if (!rng) { set_error("null rng buffer"); return TT_ERR_INVALID; }
    const int nout = (hcv != nullptr) + (scv != nullptr) + (feasible != nullptr) + (penalty != nullptr);
    if (nout != 0 && nout != 4) { set_error("evaluation outputs: all four or none"); return TT_ERR_INVALID; }
    const LsEvalOut eout{hcv, scv, feasible, penalty};
    if (max_steps < 0) { set_error("negative max_steps"); return TT_ERR_INVALID; }
    if ((rc = use_device(p))) return rc;
    const int smf = ls_mask_students(p, kMaxSlotEvents, local_search_kernel<kMaxSlotEvents>, P);
    const LsLayout Lf = ls_layout(p->E, p->R, p->dev.EW64, kMaxSlotEvents, smf);
    if (Lf.bytes > 160 * 1024) { set_error("instance too large for the local-search kernel"); return TT_ERR_LIMIT; }
    hipStream_t st = (hipStream_t)stream;
    if (order) {
        const int bits = std::min(P, kOrderCheckBits);
        hipLaunchKernelGGL(order_check_kernel, dim3(1), dim3(1024), sizeof(uint32_t) * ((bits + 31) / 32), st, order, P,
                           bits, p->dev.status);
        TT_HIP(hipGetLastError());
    }
    if (p->E <= kLsCapSmall) {                      // no slot can exceed the small tasks
        hipLaunchKernelGGL(local_search_kernel<kMaxSlotEvents>, dim3(P), dim3(64), Lf.bytes, st, p->dev, slot, room,
                           rng, P, max_steps, p1, p2, p3, (int32_t*)nullptr, 0, order, smf,
                           (unsigned long long*)nullptr, eout);
        return check_hip(hipGetLastError(), "local_search launch");
    }
    tt_problem* mp = const_cast<tt_problem*>(p);
    // the counts of this stream's call two calls back (k - 2), waited for outside the lock:
    // the masks' decision is a function of the call sequence alone
    hipEvent_t wait_ev = nullptr;
    {
        std::lock_guard<std::mutex> lock(mp->ls_mu);
        tt_problem::LsRedo* rl = find_redo(mp, stream);
        if (rl && rl->calls >= 2) wait_ev = rl->ev[rl->calls & 1];
    }
    if (wait_ev) TT_HIP(hipEventSynchronize(wait_ev));
    std::lock_guard<std::mutex> lock(mp->ls_mu);
    // this stream's redo list (grown stream-ordered: the old one may still be read)
    tt_problem::LsRedo* rl = find_redo(mp, stream);
    if (!rl) {
        mp->ls_redo.push_back({stream, nullptr, 0});
        rl = &mp->ls_redo.back();
    }
    if (!rl->ph_host) {                             // the stream's step counters (two calls' worth), once
        void* h = nullptr;
        TT_HIP(hipHostMalloc(&h, 4 * sizeof(unsigned long long), hipHostMallocDefault));
        rl->ph_host = (volatile unsigned long long*)h;
        for (int i = 0; i < 4; ++i) rl->ph_host[i] = 0ull;
    }
    for (hipEvent_t& e : rl->ev)
        if (!e) TT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (!rl->ph_dev) {
        TT_HIP(hipMallocAsync((void**)&rl->ph_dev, 2 * sizeof(unsigned long long), st));
        TT_HIP(hipMemsetAsync(rl->ph_dev, 0, 2 * sizeof(unsigned long long), st));
    }
    const int cslot = (int)(rl->calls & 1);     // this call's counter slot
    double share2 = -1.0;
    if (rl->calls >= 2) {                           // call k - 2's copy (its event waited for above)
        const unsigned long long ph2 = rl->ph_host[2 * cslot], pall = rl->ph_host[2 * cslot + 1];
        share2 = pall > 0 ? (double)ph2 / (double)pall : -1.0;
    }
    const int sms = ls_mask_students(p, kLsCapSmall, local_search_kernel<kLsCapSmall>, P, share2);
    const LsLayout Ls = ls_layout(p->E, p->R, p->dev.EW64, kLsCapSmall, sms);
    if (rl->cap < P) {
        if (rl->list) TT_HIP(hipFreeAsync(rl->list, st));
        rl->list = nullptr;
        rl->cap = 0;
        TT_HIP(hipMallocAsync((void**)&rl->list, sizeof(int32_t) * ((size_t)P + 2), st));
        TT_HIP(hipMemsetAsync(rl->list, 0, sizeof(int32_t) * 2, st));
        rl->cap = P;
    }
    hipLaunchKernelGGL(local_search_kernel<kLsCapSmall>, dim3(P), dim3(64), Ls.bytes, st, p->dev, slot, room, rng, P,
                       max_steps, p1, p2, p3, rl->list, rl->cap, order, sms, rl->ph_dev, eout);
    TT_HIP(hipGetLastError());
    // the redo launch: resident waves only (an empty list costs one short launch)
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, local_search_redo_kernel, 64, Lf.bytes) != hipSuccess) {
        (void)hipGetLastError();        // clear it: the redo launch's check below must see only its own error
        per_cu = 1;
    }
    per_cu = std::min(per_cu, lds_resident_limit(Lf.bytes));
    const int grid = std::min(P, std::max(1, per_cu) * p->num_cus);
    hipLaunchKernelGGL(local_search_redo_kernel, dim3(grid), dim3(64), Lf.bytes, st, p->dev, slot, room, rng,
                       max_steps, p1, p2, p3, rl->list, rl->cap, smf, rl->ph_dev, eout);
    const hipError_t he = hipGetLastError();
    if (he != hipSuccess) {
        // the first launch may have listed individuals: leave the list empty
        // for the stream's next call instead of redoing stale entries
        (void)hipMemsetAsync(rl->list, 0, sizeof(int32_t) * 2, st);
        return check_hip(he, "local_search redo launch");
    }
    // this call's step counts to the host for call k + 2's mask decision, then zeroed
    TT_HIP(hipMemcpyAsync((void*)(rl->ph_host + 2 * cslot), rl->ph_dev, 2 * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, st));
    TT_HIP(hipMemsetAsync(rl->ph_dev, 0, 2 * sizeof(unsigned long long), st));
    TT_HIP(hipEventRecord(rl->ev[cslot], st));
    rl->sms_last = sms;
    ++rl->calls;
    return TT_OK;
}

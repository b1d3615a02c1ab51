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
// Kernels (tt_eval_variant numbering):
//  *  8 / 7  eval_tile5 (E <= 448; 8 / 4 waves): one workgroup per tile of 64
//            individuals, a lane-per-individual phase (attendance masks) and a
//            wave-per-individual phase (bitset hcv terms) with the upper-triangle
//            correlation words resident in registers;
//  * 13      the wide path (E > 448): eval_lanes (the lane phase over a 64-row
//            tile, 16 waves) + eval_corr (the hcv terms for batches of
//            individuals; each wave keeps the correlation words of a pair of
//            64-event chunks in registers for the whole launch);
//  *  2      eval_block (any E): one 256-thread workgroup per individual.
#include <algorithm>
#include <type_traits>
#include <utility>
#include <vector>

#include "tt_internal.h"

namespace ttga {

typedef __attribute__((address_space(4))) const uint32_t ConstU32;
typedef __attribute__((address_space(4))) const int32_t ConstI32;

// ---------------------------------------------------------------- eval_tile5
// TT_T5_ROOMBUF: slot-row DMA and room rows by buffer instructions (per-tile
// resource, 32-bit lane offsets): no 64-bit per-lane pointer lives across the
// tile loop (it spilled to scratch: 8 B per thread per tile, 4 MB per launch at
// P = 65,536).
#ifndef TT_T5_ROOMBUF
#define TT_T5_ROOMBUF 1
#endif
// NW waves per 64-individual tile; one tile per workgroup (the loop also runs a
// persistent grid). Slot rows are staged by LDS-DMA (DB: two tile buffers, the
// next tile of a persistent grid lands under the current one's evaluation).
//  * lane phase (LANE = INDIVIDUAL): per-student records of 8 u16 event ids
//    (padded with the sentinel column E = slot 63, end-of-student flag in bit
//    15) come through the scalar cache (s_load_dwordx4 via the constant
//    address space) from a student-ordered stream; wave w owns a contiguous
//    student range balanced by record count; 8 conflict-free ds_read_u8 per
//    record from the tile (odd-dword row stride) build the 45-bit attendance
//    mask -> >2-in-a-row and single-class terms. A back-to-back record stream
//    with per-entry end flags measured slower: its uniform per-entry branches
//    serialise the mask updates;
//  * wave phase (WAVE = INDIVIDUAL): slot rows from the tile, room rows from
//    global memory one individual ahead; per-slot event bitsets B[t]
//    (ds_or_b64), room-cell counters (packed u16, ds_add_rtn), unsuitable
//    rooms, last-slot term, and the correlated same-slot pairs as
//    popcount(cupT[w][i] & B[slot_i][w]) over the upper-triangle words, which
//    (with possibleRooms and studentNumber) stay in registers for the launch;
//  * an individual with an invalid gene is detected from registers before any
//    LDS work (its outputs are the -1 sentinels); the valid path has no
//    per-event branches except on the last, partial event word;
//  * PK: 1 = possibleRooms | studentNumber << 16 in one register (R <= 16,
//    studentNumber < 65536), 2 = u32 mask (R <= 32), 0 = u64 mask.

// acc + popcount(x) as two v_bcnt_u32_b32 with accumulate (no separate add).
// (The compiler turns the plain form into bcnt, bcnt, add3.)
__device__ __forceinline__ int bcnt_acc(uint32_t x, int acc) {
    int r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}
__device__ __forceinline__ int popc_acc(uint64_t x, int acc) {
    int r, t;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(t) : "v"((uint32_t)x), "v"(acc));
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"((uint32_t)(x >> 32)), "v"(t));
    return r;
}

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

// NA consecutive 64-bit LDS words at byte address a and NB at b (NA + NB <= 8),
// all in flight at once, waited for inside the asm.
#define TT_O(k) [d##k] "=&v"(d[k])
#define TT_I(k) [x##k] "v"(k < NA ? a : b), [o##k] "i"(k < NA ? 8 * k : 8 * (k - NA))
#define TT_R(k) "ds_read_b64 %[d" #k "], %[x" #k "] offset:%[o" #k "]\n"
template <int NA, int NB>
__device__ __forceinline__ void lds_two_rows(uint32_t a, uint32_t b, uint64_t* v) {
    constexpr int N = NA + NB;
    static_assert(NA >= 1 && NB >= 0 && N <= 8, "1..8 words");
    uint64_t d[8];
    if constexpr (N == 8)
        asm volatile(TT_R(0) TT_R(1) TT_R(2) TT_R(3) TT_R(4) TT_R(5) TT_R(6) TT_R(7) "s_waitcnt lgkmcnt(0)"
                     : TT_O(0), TT_O(1), TT_O(2), TT_O(3), TT_O(4), TT_O(5), TT_O(6), TT_O(7)
                     : TT_I(0), TT_I(1), TT_I(2), TT_I(3), TT_I(4), TT_I(5), TT_I(6), TT_I(7) : "memory");
    else if constexpr (N == 7)
        asm volatile(TT_R(0) TT_R(1) TT_R(2) TT_R(3) TT_R(4) TT_R(5) TT_R(6) "s_waitcnt lgkmcnt(0)"
                     : TT_O(0), TT_O(1), TT_O(2), TT_O(3), TT_O(4), TT_O(5), TT_O(6)
                     : TT_I(0), TT_I(1), TT_I(2), TT_I(3), TT_I(4), TT_I(5), TT_I(6) : "memory");
    else if constexpr (N == 6)
        asm volatile(TT_R(0) TT_R(1) TT_R(2) TT_R(3) TT_R(4) TT_R(5) "s_waitcnt lgkmcnt(0)"
                     : TT_O(0), TT_O(1), TT_O(2), TT_O(3), TT_O(4), TT_O(5)
                     : TT_I(0), TT_I(1), TT_I(2), TT_I(3), TT_I(4), TT_I(5) : "memory");
    else if constexpr (N == 5)
        asm volatile(TT_R(0) TT_R(1) TT_R(2) TT_R(3) TT_R(4) "s_waitcnt lgkmcnt(0)"
                     : TT_O(0), TT_O(1), TT_O(2), TT_O(3), TT_O(4) : TT_I(0), TT_I(1), TT_I(2), TT_I(3), TT_I(4) : "memory");
    else if constexpr (N == 4)
        asm volatile(TT_R(0) TT_R(1) TT_R(2) TT_R(3) "s_waitcnt lgkmcnt(0)"
                     : TT_O(0), TT_O(1), TT_O(2), TT_O(3) : TT_I(0), TT_I(1), TT_I(2), TT_I(3) : "memory");
    else if constexpr (N == 3)
        asm volatile(TT_R(0) TT_R(1) TT_R(2) "s_waitcnt lgkmcnt(0)"
                     : TT_O(0), TT_O(1), TT_O(2) : TT_I(0), TT_I(1), TT_I(2) : "memory");
    else if constexpr (N == 2)
        asm volatile(TT_R(0) TT_R(1) "s_waitcnt lgkmcnt(0)" : TT_O(0), TT_O(1) : TT_I(0), TT_I(1) : "memory");
    else
        asm volatile(TT_R(0) "s_waitcnt lgkmcnt(0)" : TT_O(0) : TT_I(0) : "memory");
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = d[k];
}
#undef TT_O
#undef TT_I
#undef TT_R

// Correlated same-slot pairs of the lane's events:
// h += popcount(cupT upper words & B[slot] words). Event words R and EWC-1-R
// are read together (EWC+1 row words in one asm block): ceil(EWC/2) LDS round
// trips per individual instead of EWC.
template <int R, int EWC>
__device__ __forceinline__ void corr_words(uint32_t bbase, const uint32_t* sv, const uint64_t (*cup)[EWC], int lane,
                                           int E, bool last_partial, int& h) {
    constexpr int S = EWC - 1 - R;                     // partner word
    if constexpr (R < S) {
        // word S may be the last, partial one: its lanes beyond E read row 0 (harmless,
        // their cup words are zero)
        const uint32_t ss = (S < EWC - 1 || !last_partial || lane + 64 * S < E) ? sv[S] : 0u;
        uint64_t bw[EWC + 1];
        lds_two_rows<EWC - R, EWC - S>(bbase + sv[R] * (uint32_t)(EWC * 8) + 8 * R,
                                       bbase + ss * (uint32_t)(EWC * 8) + 8 * S, bw);
#pragma unroll
        for (int w = R; w < EWC; ++w) h = popc_acc(cup[R][w] & bw[w - R], h);
#pragma unroll
        for (int w = S; w < EWC; ++w) h = popc_acc(cup[S][w] & bw[EWC - R + w - S], h);
        corr_words<R + 1, EWC>(bbase, sv, cup, lane, E, last_partial, h);
    } else if constexpr (R == S) {
        if (R < EWC - 1 || !last_partial || lane + 64 * R < E) {
            uint64_t bw[EWC - R];
            lds_row_b64<EWC - R>(bbase + sv[R] * (uint32_t)(EWC * 8) + 8 * R, bw);
#pragma unroll
            for (int w = R; w < EWC; ++w) h = popc_acc(cup[R][w] & bw[w - R], h);
        }
    }
}

// ---------------------------------------------------------------- scalar record loads
// Records come through the scalar cache by the compiler's own s_load (uniform
// index into the constant address space), so it tracks every load and places
// the s_waitcnt itself. (Round 4 issued them from inline asm with a separate
// wait; the compiler could copy the destination registers between issue and
// wait -- a data race that showed up once as nondeterministic wide-path
// results. tests/test_codeobj.py::test_no_inline_asm_scalar_loads_in_sources checks the
// built code object for asm-issued scalar loads.)
template <int ST>
__device__ __forceinline__ void sload_rec(const ConstU32* q, uint32_t (&r)[ST]) {
#pragma unroll
    for (int j = 0; j < ST; ++j) r[j] = q[j];
}
// An empty use of a prefetched record after the step that overlaps it: the
// load cannot then be sunk into the next step (where its wait would expose the
// whole scalar-cache latency); the step's own LDS wait, lgkmcnt(0), has already
// covered it, so the use costs no wait.
template <int ST>
__device__ __forceinline__ void keep_rec(const uint32_t (&r)[ST]) {
#pragma unroll
    for (int j = 0; j < ST; ++j) asm volatile("" ::"s"(r[j]));
}

// ---------------------------------------------------------------- student runs
// The lane phase over the size-sorted student lists (DevProblem::sid/srun):
// a run holds `cnt` students of N ids each (N even, the last id may be the
// sentinel E), so a student costs its own events plus at most one sentinel.
// mask_scv (>2 in a row + single class of one student's mask): tt_common.h
// The same terms for a mask in the GAPPED slot layout of eval_lanes' tile
// (TT_LANES_GAP): slot s = 9d + k sits at bit 10d + k for days 0-2 and at bit
// 32 + 10(d - 3) + k for days 3-4, so every day is a 9-bit field followed by a
// zero bit and no field straddles the 32-bit halves (the tile's sentinel
// column keeps bit 63). Then:
//  * >2 in a row: m & m>>1 & m>>2 cannot cross a day (the zero bit), no mask;
//  * single class, per half, every field f at once: b = x + K (K = 511 per
//    field, no carry out of a field) has the field's top bit set iff f != 0 and
//    its low bits f - 1, so t = x & b is f & (f - 1) per field, and
//    [popcount(f) == 1] = top bit of b and not of t + K. 14 VALU for the five
//    days instead of 21 (bfe, bcnt, compare, add per day).
constexpr uint32_t kGapLoK = 0x1FF7FDFFu, kGapLoG = 0x20080200u;    // fields at bits 0, 10, 20
constexpr uint32_t kGapHiK = 0x0007FDFFu, kGapHiG = 0x00080200u;    // fields at bits 32, 42
__device__ __forceinline__ int mask_scv_gap(uint64_t m) {
    int sc = __popcll(m & (m >> 1) & (m >> 2));
    const uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
    const uint32_t blo = lo + kGapLoK, bhi = hi + kGapHiK;
    const uint32_t tlo = (lo & blo) + kGapLoK, thi = (hi & bhi) + kGapHiK;
    sc += __popc((blo ^ tlo) & kGapLoG);
    sc += __popc((bhi ^ thi) & kGapHiG);
    return sc;
}
// slot bytes -> gapped bit positions, four bytes of one row at a time (valid
// slots < 45; a byte >= 128 of an invalid genome may spill into its row
// neighbour, whose individual evaluates to the invalid sentinel anyway):
// p = s + [s >= 9] + [s >= 18] + 3 [s >= 27] + [s >= 36]
__device__ __forceinline__ uint32_t gap_slots4(uint32_t x) {
    const uint32_t o = x | 0x80808080u;
    const uint32_t g9 = ((o - 0x09090909u) >> 7) & 0x01010101u, g18 = ((o - 0x12121212u) >> 7) & 0x01010101u;
    const uint32_t g27 = ((o - 0x1B1B1B1Bu) >> 7) & 0x01010101u, g36 = ((o - 0x24242424u) >> 7) & 0x01010101u;
    return x + g9 + g18 + g36 + 3u * g27;
}
__device__ __forceinline__ uint8_t gap_slot(uint32_t s) { return (uint8_t)gap_slots4(s); }
#ifndef TT_LANES_GAP
#define TT_LANES_GAP 1
#endif
template <bool GAP>
__device__ __forceinline__ int mask_terms(uint64_t m) { return GAP ? mask_scv_gap(m) : mask_scv(m); }
// K students of N ids whose dwords are r[0 .. K*N/2)
template <int N, int K, bool GAP = false>
__device__ __forceinline__ int students_scv(const uint8_t* my, const uint32_t* r) {
    constexpr int H = N / 2;
    uint32_t sl[K * N];
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int j = 0; j < N; ++j) sl[k * N + j] = my[(r[k * H + (j >> 1)] >> (16 * (j & 1))) & 0xFFFFu];
    int sc = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint64_t m = 0;
#pragma unroll
        for (int j = 0; j < N; ++j) m |= 1ull << (sl[k * N + j] & 63);
        sc += mask_terms<GAP>(m);
    }
    return sc;
}
// A run of cnt students of N ids from dword p: one scalar load of K*N/2
// dwords per step (K = 2 students when N <= 16), the next step's load issued
// before this step's LDS reads (ping-pong registers, no copies).
template <int N, int KMAX, bool GAP = false>
__device__ __forceinline__ int run_scv(const uint8_t* my, const uint32_t* p, int cnt) {
    constexpr int K = N <= 16 ? KMAX : 1;
    constexpr int ST = K * N / 2;
    const int steps = cnt / K;
    int sc = 0;
    if constexpr (KMAX == 1) {
        // one student per step, its ids through the compiler's scalar loads
        // with the next student's issued ahead (fewer SGPRs than ping-pong)
        const ConstU32* q = (const ConstU32*)p;
        uint32_t cur[N / 2];
#pragma unroll
        for (int j = 0; j < N / 2; ++j) cur[j] = q[j];
        for (int i = 0; i < cnt; ++i) {
            const int in = i + 1 < cnt ? i + 1 : i;
            uint32_t nxt[N / 2];
#pragma unroll
            for (int j = 0; j < N / 2; ++j) nxt[j] = q[in * (N / 2) + j];
            uint32_t sl[N];
#pragma unroll
            for (int j = 0; j < N; ++j) sl[j] = my[(cur[j >> 1] >> (16 * (j & 1))) & 0xFFFFu];
            uint64_t m = 0;
#pragma unroll
            for (int j = 0; j < N; ++j) m |= 1ull << (sl[j] & 63);
            sc += mask_terms<GAP>(m);
#pragma unroll
            for (int j = 0; j < N / 2; ++j) cur[j] = nxt[j];
        }
        return sc;
    }
    const ConstU32* q = (const ConstU32*)p;
    if (steps > 0) {
        int i = 0;
        uint32_t ra[ST], rb[ST];
        sload_rec<ST>(q, ra);
        while (true) {
            sload_rec<ST>(q + (i + 1 < steps ? i + 1 : i) * ST, rb);
            sc += students_scv<N, K, GAP>(my, ra);
            keep_rec<ST>(rb);
            if (++i == steps) break;
            sload_rec<ST>(q + (i + 1 < steps ? i + 1 : i) * ST, ra);
            sc += students_scv<N, K, GAP>(my, rb);
            keep_rec<ST>(ra);
            if (++i == steps) break;
        }
    }
    if constexpr (K == 2) {
        if (cnt & 1) {
            uint32_t r[N / 2];
            sload_rec<N / 2>(q + steps * ST, r);
            sc += students_scv<N, 1, GAP>(my, r);
        }
    }
    return sc;
}
// students of more than 32 ids (no instance here has them): plain loop
__device__ __noinline__ int run_scv_any(const uint8_t* my, const ConstU32* p, int cnt, int n, bool gap) {
    int sc = 0;
    for (int i = 0; i < cnt; ++i) {
        uint64_t m = 0;
        for (int j = 0; j < n / 2; ++j) {
            const uint32_t d = p[i * (n / 2) + j];
            m |= 1ull << (my[d & 0xFFFFu] & 63);
            m |= 1ull << (my[d >> 16] & 63);
        }
        sc += gap ? mask_scv_gap(m) : mask_scv(m);
    }
    return sc;
}
template <int KMAX, bool GAP = false>
__device__ __forceinline__ int lane_scv_runs(const uint8_t* my, const DevProblem& pb, int r0, int r1) {
    const ConstI32* runs = (const ConstI32*)pb.srun;
    int sc = 0;
    for (int k = r0; k < r1; ++k) {
        const int n = runs[4 * k], off = runs[4 * k + 1], cnt = runs[4 * k + 2];
        const uint32_t* p = pb.sid + off;
        switch (n) {
#define TT_RUN(N) case N: sc += run_scv<N, KMAX, GAP>(my, p, cnt); break;
            TT_RUN(2) TT_RUN(4) TT_RUN(6) TT_RUN(8) TT_RUN(10) TT_RUN(12) TT_RUN(14) TT_RUN(16)
            TT_RUN(18) TT_RUN(20) TT_RUN(22) TT_RUN(24) TT_RUN(26) TT_RUN(28) TT_RUN(30) TT_RUN(32)
#undef TT_RUN
            default: sc += run_scv_any(my, (const ConstU32*)p, cnt, n, GAP); break;
        }
    }
    return sc;
}

// Per-event phase ablations (tt_eval_variant's profiling bits 4..32) are compiled
// in only with -DTT_EVAL_ABLATE=1: as runtime flags they put a uniform branch
// around every per-event atomic, which also serialises each cell-counter
// return. Bits 1 and 2 (skip the lane / wave phase: once per tile or batch)
// stay, for bench.py's FETCH_SIZE calibration pass (staging and outputs only).
#ifndef TT_EVAL_ABLATE
#define TT_EVAL_ABLATE 0
#endif
// Cell counters of eval_tile5 (TT_T5_CELLS = 1): [45][RW] dwords, RW = ceil(R/2),
// cell (s, ro) in dword s*RW + ro/2, half ro & 1 -- fewer address instructions
// than the packed cell index (s*R + ro)/2.
#ifndef TT_T5_CELLS
#define TT_T5_CELLS 1
#endif
__host__ __device__ inline int t5_cnt_bytes(int R) {
#if TT_T5_CELLS
    return kSlots * ((R + 1) / 2) * 4;
#else
    return ((kSlots * R + 1) / 2) * 4;
#endif
}

struct Tile5Layout {
    int SP, WS;
    size_t tile_bytes, off_ws, off_part, bytes;
};

// DB: two tile buffers; the next tile's slot rows land by LDS-DMA while the
// current one is evaluated.
__host__ __device__ inline Tile5Layout tile5_layout(int E, int R, int NW, bool DB = false) {
    Tile5Layout L;
    int sp = (E + 1 + 3) & ~3;                 // room for the sentinel column
    if (((sp >> 2) & 1) == 0) sp += 4;         // odd dword stride: conflict-free column reads
    L.SP = sp;
    const int ew64 = (E + 63) / 64;
    const int cntb = t5_cnt_bytes(R);
    L.WS = (kSlots * ew64 * 8 + cntb + 15) & ~15;
    L.tile_bytes = ((size_t)64 * sp + 15) & ~(size_t)15;
    L.off_ws = (DB ? 2 : 1) * L.tile_bytes;
    L.off_part = L.off_ws + (size_t)NW * L.WS;
    L.bytes = L.off_part + 4 * (size_t)(NW * 64 + 64);
    return L;
}

// One wave's share of a tile's slot rows by LDS-DMA (global_load_lds_dword:
// 64 lanes x 4 B land contiguously at a wave-uniform LDS address, so a row of
// E/4 <= 112 dwords takes two instructions and keeps its padded stride SP).
// Buffer-load form (TT_T5_ROOMBUF): a per-tile resource, a 32-bit lane offset
// and a scalar row offset (the global form kept a 64-bit per-lane pointer live
// across the tile loop, which spilled to scratch).
template <int NW>
__device__ __forceinline__ void tile_dma(const uint8_t* src, uint8_t* dst, int np, int E, int SP, int wv, int lane) {
    const int qd = E >> 2;
#if TT_T5_ROOMBUF
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, np * E, 0x00020000);
    for (int r = wv; r < np; r += NW) {
        if (lane < qd)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + r * SP), 4,
                                                     4 * lane, r * E, 0, 0);
        if (lane + 64 < qd)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + r * SP + 256),
                                                     4, 4 * lane + 256, r * E, 0, 0);
    }
#else
    for (int r = wv; r < np; r += NW) {
        const uint32_t* g = (const uint32_t*)(src + (long)r * E);
        auto* d = (__attribute__((address_space(3))) void*)(dst + r * SP);
        if (lane < qd)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + lane), d, 4, 0, 0);
        if (lane + 64 < qd)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + 64 + lane),
                                             (__attribute__((address_space(3))) void*)(dst + r * SP + 256), 4, 0, 0);
    }
#endif
}

// Profiling build (-DTT_T5_STAMP, libttga_prof.so, tools/t5_stamps.py): per
// workgroup, the constant-clock time (s_memrealtime, 100 MHz) when its wave 0
// starts and when each of its waves ends, and the hardware slot it ran on
// (HW_ID, XCC_ID), for launch index (variant bits 12..14) of kT5Launches. No
// atomics and no extra barrier: the stamps cost a few stores per wave.
#ifdef TT_T5_STAMP
constexpr int kT5Launches = 8, kT5MaxBlocks = 16384, kT5Words = 10;   // t0, id, end of waves 0..7
__device__ unsigned long long g_t5_stamp[kT5Launches * kT5MaxBlocks * kT5Words];
#endif

// a.lo16 * b.hi16 + c in one VALU instruction (v_mad_u32_u16, op_sel on src1)
__device__ __forceinline__ uint32_t mad_u16_hi(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_mad_u32_u16 %0, %1, %2, %3 op_sel:[0,1,0,0]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// TT_T5_PRIO: issue priority falls as a wave gets through its tile (3 in the
// lane phase, then 3, 3, 2, 2, 1, 1, 0, 0 over its wave-phase individuals), so
// of a CU's two resident workgroups the one further behind wins the arbiter --
// instead of the older one (round-4 stamps: the older finishes 31.9 us, its
// neighbour 43.0 us, and the CU's last workgroup runs alone for 15 us). Same
// box (profiles/r05_ab_tile5_prio.jsonl): med 74.2 -> 71.8 us, lg 96.9 -> 94.1,
// comp01 100.0 -> 100.1; slower decays measured 72.1-73.1 us at med.
#ifndef TT_T5_PRIO
#define TT_T5_PRIO 1
#endif
// the schedule: priority in the lane phase, then per individual i of the wave's
// (up to 8) wave-phase individuals nibble i of TT_T5_PRIO_W
#ifndef TT_T5_PRIO_LANE
#define TT_T5_PRIO_LANE 3
#endif
#ifndef TT_T5_PRIO_W
#define TT_T5_PRIO_W 0x00112233u
#endif
template <int EWC, int NW, int PK, bool DB = false>
__global__ __launch_bounds__(64 * NW, 4) void eval_tile5_kernel(DevProblem pb, const uint8_t* __restrict__ slot,
                                                              const uint8_t* __restrict__ room, int P,
                                                              int32_t* __restrict__ hcv_out,
                                                              int32_t* __restrict__ scv_out,
                                                              uint8_t* __restrict__ feas_out,
                                                              int32_t* __restrict__ pen_out, int ablate_arg) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int ablate = TT_EVAL_ABLATE ? ablate_arg : (ablate_arg & 3);   // phase skips: once per tile / batch
    constexpr int NT = 64 * NW;
#ifdef TT_T5_STAMP
    unsigned long long* st_rec =
        g_t5_stamp + ((size_t)((ablate_arg >> 8) & (kT5Launches - 1)) * kT5MaxBlocks + (blockIdx.x % kT5MaxBlocks)) * kT5Words;
    if (threadIdx.x == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        st_rec[0] = t0;
        st_rec[1] = ((unsigned long long)xcc << 32) | hw;
    }
#endif
    const int E = pb.E, R = pb.R;
    const int lane = threadIdx.x & 63, wv = wave_id();
    const Tile5Layout L = tile5_layout(E, R, NW, DB);
    const int SP = L.SP;
    uint8_t* tile = lds;
    uint8_t* ws = lds + L.off_ws + (size_t)wv * L.WS;
    uint64_t* B = (uint64_t*)ws;                              // [45][EWC] event bitsets per slot
    uint32_t* cnt = (uint32_t*)(B + kSlots * EWC);            // packed u16 cell counters
    int32_t* part = (int32_t*)(lds + L.off_part);             // [NW][64] scv partials
    int32_t* hq = part + NW * 64;                             // [64] hcv (or -1)
    const int tiles = (P + 63) / 64;
    const bool last_partial = E < 64 * EWC;                   // lanes of word EWC-1 beyond E
    const int RW = (R + 1) / 2;

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
            // low half: the rooms NOT possible for e (one bfe gives the unsuitable-room
            // term), high half: studentNumber (read by v_mad_u32_u16's op_sel)
            inv_ps[r] = ok ? ((~(uint32_t)pb.poss[e] & 0xFFFFu) | ((uint32_t)pb.sn[e] << 16)) : 0u;
        } else {
            inv_poss[r] = ok ? (PossT)pb.poss[e] : (PossT)~0ull;
            inv_sn[r] = ok ? pb.sn[e] : 0;
        }
#pragma unroll
        for (int w = 0; w < EWC; ++w) inv_cup[r][w] = (w >= r && ok) ? pb.cupT[(size_t)w * E + e] : 0ull;
    }
    const ConstI32* ptab = (const ConstI32*)pb.srun_part;
    const int pbase = srun_part_base(NW);
    const int r0 = ptab[pbase + wv], r1 = ptab[pbase + wv + 1];     // this wave's student runs
    const bool wide = (E & 15) == 0 && (((uintptr_t)slot) & 15) == 0;
    const int qpr = E >> 4;
    const uint32_t qinv = ((1u << 20) + (uint32_t)qpr - 1) / (uint32_t)max(qpr, 1);

    if constexpr (DB) {
        // sentinel columns of both buffers (the DMA writes columns < E only), then the first tile
        if (threadIdx.x < 128) lds[(threadIdx.x >> 6) * L.tile_bytes + (threadIdx.x & 63) * SP + E] = 63;
        if (blockIdx.x < tiles)
            tile_dma<NW>(slot + (long)blockIdx.x * 64 * E, lds, (int)min(64L, (long)P - (long)blockIdx.x * 64), E, SP,
                         wv, lane);
    }
    int it = 0;
    for (int tl = blockIdx.x; tl < tiles; tl += gridDim.x, ++it) {
        const long p0 = (long)tl * 64;
        const int np = (int)min((long)64, (long)P - p0);
        const uint8_t* src = slot + p0 * E;
        if constexpr (DB) {
            tile = lds + (it & 1) * L.tile_bytes;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // this wave's DMAs of the tile
            __syncthreads();                                       // everyone's; the other buffer is free
            const int tn = tl + gridDim.x;
            if (tn < tiles)
                tile_dma<NW>(slot + (long)tn * 64 * E, lds + ((it + 1) & 1) * L.tile_bytes,
                             (int)min(64L, (long)P - (long)tn * 64), E, SP, wv, lane);
        } else {
        __syncthreads();
        // ---- stage the tile's slot rows (+ sentinel column E = slot 63)
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
        }

        // ---- lane phase (lane = individual): attendance masks of this wave's students
        // lane * SP recomputed per tile (an asm multiply the compiler cannot hoist:
        // kept live across the tile loop, the product spilled to scratch)
        uint32_t lsp;
        asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(lsp) : "v"(lane), "s"(SP));
        if (TT_T5_PRIO) __builtin_amdgcn_s_setprio(TT_T5_PRIO_LANE);
        const int sc = (!(ablate & 1) && r0 < r1) ? lane_scv_runs<1>(tile + lsp, pb, r0, r1) : 0;
        part[wv * 64 + lane] = sc;

        // ---- wave phase (wave = individual): hcv terms + last-slot term
        const int nq = (ablate & 2) ? 0 : np;
        uint32_t pfn[EWC];                                        // room row, one individual ahead
#if TT_T5_ROOMBUF
        // room rows by buffer loads from a per-tile resource: a 32-bit lane offset
        // and a scalar row offset instead of a 64-bit per-lane pointer kept live
        // across the tile loop (it spilled to scratch: 8 B per thread per tile)
        const __amdgpu_buffer_rsrc_t rrs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(room + p0 * E), 0, 64 * E, 0x00020000);
        auto load_row = [&](const uint8_t*, int q, uint32_t* dst) {
#pragma unroll
            for (int r = 0; r < EWC; ++r)
                dst[r] = (!last_partial || r < EWC - 1 || lane + 64 * r < E)
                             ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rrs, lane + 64 * r, q * E, 0)
                             : 0u;
        };
#else
        auto load_row = [&](const uint8_t* base, int q, uint32_t* dst) {
            const uint8_t* rr = base + (p0 + q) * E;
#pragma unroll
            for (int r = 0; r < EWC; ++r)
                dst[r] = (!last_partial || r < EWC - 1 || lane + 64 * r < E) ? rr[lane + 64 * r] : 0u;
        };
#endif
        if (wv < nq) load_row(room, wv, pfn);
        for (int q = wv; q < nq; q += NW) {
            if (TT_T5_PRIO) {
                // s_setprio takes an immediate: one of four, by the schedule's nibble
                const uint32_t pr = (TT_T5_PRIO_W >> (4 * min((q - wv) / NW, 7))) & 3u;
                if (pr == 0) __builtin_amdgcn_s_setprio(0);
                else if (pr == 1) __builtin_amdgcn_s_setprio(1);
                else if (pr == 2) __builtin_amdgcn_s_setprio(2);
                else __builtin_amdgcn_s_setprio(3);
            }
            uint32_t rv[EWC], sv[EWC];
#pragma unroll
            for (int r = 0; r < EWC; ++r) rv[r] = pfn[r];
            const uint8_t* rs = tile + q * SP;
#pragma unroll
            for (int r = 0; r < EWC; ++r)
                sv[r] = (!last_partial || r < EWC - 1 || lane + 64 * r < E) ? rs[lane + 64 * r] : 0u;
            if (q + NW < nq) load_row(room, q + NW, pfn);             // next individual
            // an invalid gene anywhere -> sentinel outputs; decided from registers
            uint32_t smax = 0, rmax = 0;
#pragma unroll
            for (int r = 0; r < EWC; ++r) { smax = max(smax, sv[r]); rmax = max(rmax, rv[r]); }
            const bool any_bad = wave_any(smax >= (uint32_t)kSlots || rmax >= (uint32_t)R);
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
                        if (!(ablate & 16)) {                                   // Solution.cpp:148-150
#if TT_T5_CELLS
                            // dword s*RW + ro/2: byte offset 2*(s*2RW + (ro & ~1))
                            uint32_t* c = (uint32_t*)((uint8_t*)cnt + ((__umul24(s, (uint32_t)(2 * RW)) + (ro & ~1u)) << 1));
                            const uint32_t sh = ro << 4;                        // shifts and bfe use bits 4:0
                            // (v_bfe_u32 reads offset bits 4:0, as the shift does)
                            h += (int)__builtin_amdgcn_ubfe(atomicAdd(c, 1u << (sh & 31u)), sh, 16);
#else
                            const uint32_t cell = s * (uint32_t)R + ro;
                            const uint32_t sh = (cell & 1u) << 4;
                            h += (int)((atomicAdd(&cnt[cell >> 1], 1u << sh) >> sh) & 0xFFFFu);
#endif
                        }
                        const bool last_slot = (kLastSlotMask >> s) & 1ull;
                        if constexpr (PK == 1) {
                            h += (int)__builtin_amdgcn_ubfe(inv_ps[r], ro, 1);               // :155-156
#if TT_T5_CELLS
                            last = (int)mad_u16_hi((uint32_t)(kLastSlotMask >> s) & 1u, inv_ps[r], (uint32_t)last);   // :93-96
#else
                            last += last_slot ? (int)(inv_ps[r] >> 16) : 0;             // :93-96 (unused: PK 1 with TT_T5_CELLS)
#endif
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
                // one reduction of h << 16 | last when every lane's two parts are < 1024
                // (so both 64-lane sums stay below 2^16), else two
                if (!wave_any(h >= 1024 || last >= 1024)) {
                    const uint32_t t = (uint32_t)wave_sum((h << 16) | last);
                    h = (int)(t >> 16);
                    last = (int)(t & 0xFFFFu);
                } else {
                    h = wave_sum(h);
                    last = wave_sum(last);
                }
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
#ifdef TT_T5_STAMP
    if ((threadIdx.x & 63) == 0 && (threadIdx.x >> 6) < kT5Words - 2)
        st_rec[2 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memrealtime();
#endif
}

// ---------------------------------------------------------------- eval_lanes
// The lane phase of eval_tile5 on its own (wide path, E > 448): a 16-wave
// workgroup per 64-row tile (128 KB at E = 2000: one workgroup per CU); it
// writes the per-student scv part (>2 in a row + single class) of each
// individual to scv_part, which eval_corr completes.
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
    const ConstI32* ptab = (const ConstI32*)pb.srun_part;
    const int pbase = srun_part_base(NWL);
    const int r0 = ptab[pbase + wv], r1 = ptab[pbase + wv + 1];     // this wave's student runs
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
                if (TT_LANES_GAP) {
                    d[0] = gap_slots4(v.x); d[1] = gap_slots4(v.y); d[2] = gap_slots4(v.z); d[3] = gap_slots4(v.w);
                } else {
                    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
                }
            }
        } else {
#pragma unroll 1
            for (int r = wv; r < np; r += NWL)
#pragma unroll 1
                for (int c = lane; c < E; c += 64) {
                    const uint8_t v = src[(long)r * E + c];
                    tile[r * SP + c] = TT_LANES_GAP ? gap_slot(v) : v;
                }
        }
        if (threadIdx.x < 64) tile[threadIdx.x * SP + E] = 63;
        __syncthreads();
        const int sc = r0 < r1 ? lane_scv_runs<2, TT_LANES_GAP != 0>(tile + lane * SP, pb, r0, r1) : 0;
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

// ---------------------------------------------------------------- eval_corr
// The hcv terms (and the last-slot scv term) of the wide path, after
// eval_lanes. The upper-triangle correlation stream (E x EW64 / 2 u64 words,
// 264 KB at E = 2000) is the same for every individual, so a workgroup reads
// it once per batch of NB individuals instead of once per individual:
//  * build phase: wave v owns EPL consecutive events per lane (their
//    possibleRooms / studentNumber stay in registers) and, for every
//    individual of the batch, sets the slot bitsets B_q[45][BST] (ds_or_b64),
//    counts room cells in packed u16 counters (ds_add_rtn: the returned old
//    counts sum to sum_cells C(n,2)), adds unsuitable rooms and the last-slot
//    term and stages the slot row in LDS;
//  * corr phase: the 64-event chunks are taken in pairs (a, EW64-1-a), so
//    every pair has EW64+1 upper-triangle words per event; wave v streams the
//    words w >= c of its chunks' events (coalesced 512-B loads, four words
//    ahead) and, for each word, gathers B_q[slot][w] of all NB individuals
//    (NB independent ds_read_b64 in flight) and adds popcount(word & B word).
// Per-individual LDS: B rows (odd u64 stride BST = EW64 | 1), counters, slot row.
//   hcv  = sum over cells of C(n, 2)                (Solution.cpp:148-150)
//        + sum_e [room_e not possible]              (:155-156)
//        + sum_e sum_{w >= e/64} popcount(cupT[w][e] & B[slot_e][w])   (:151-153)
//   scv += sum_e [slot_e % 9 == 8] studentNumber[e] (:93-96)
struct CorrLayout {
    int NWV, BST, NB, EPL;
    size_t off_cnt, off_sl, WSI, off_acc, off_red, bytes;
};

__host__ __device__ inline CorrLayout corr_layout(int E, int R, int EW64, int NB) {
    CorrLayout L;
    const int pairs = (EW64 + 1) / 2;
    L.NWV = pairs < 16 ? pairs : 16;
    L.EPL = (E + 64 * L.NWV - 1) / (64 * L.NWV);
    L.BST = EW64 | 1;
    L.off_cnt = (size_t)kSlots * L.BST * 8;
    L.off_sl = L.off_cnt + (size_t)((kSlots * R + 1) / 2) * 4;
    L.WSI = (L.off_sl + (size_t)E + 15) & ~(size_t)15;
    L.NB = NB;
    L.off_acc = (size_t)NB * L.WSI;
    L.off_red = L.off_acc + (size_t)NB * 16;
    L.bytes = L.off_red + (size_t)NB * 2 * 64 * 4;
    return L;
}

constexpr int kCorrMaxEPL = 4;

// N ds_read_b64 at N per-lane byte addresses + OFF, all in flight at once,
// waited for inside the asm (results defined when it ends).
template <int N, int OFF>
__device__ __forceinline__ void lds_gather(const uint32_t* a, uint64_t* v) {
    static_assert(N == 2 || N == 4 || N == 8, "2, 4 or 8 reads");
    if constexpr (N == 8)
        asm volatile("ds_read_b64 %0, %8 offset:%16\n ds_read_b64 %1, %9 offset:%16\n ds_read_b64 %2, %10 offset:%16\n"
                     "ds_read_b64 %3, %11 offset:%16\n ds_read_b64 %4, %12 offset:%16\n ds_read_b64 %5, %13 offset:%16\n"
                     "ds_read_b64 %6, %14 offset:%16\n ds_read_b64 %7, %15 offset:%16\n s_waitcnt lgkmcnt(0)"
                     : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
                     : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "i"(OFF)
                     : "memory");
    else if constexpr (N == 4)
        asm volatile("ds_read_b64 %0, %4 offset:%8\n ds_read_b64 %1, %5 offset:%8\n ds_read_b64 %2, %6 offset:%8\n"
                     "ds_read_b64 %3, %7 offset:%8\n s_waitcnt lgkmcnt(0)"
                     : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
                     : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "i"(OFF) : "memory");
    else
        asm volatile("ds_read_b64 %0, %2 offset:%4\n ds_read_b64 %1, %3 offset:%4\n s_waitcnt lgkmcnt(0)"
                     : "=&v"(v[0]), "=&v"(v[1]) : "v"(a[0]), "v"(a[1]), "i"(OFF) : "memory");
}

// Words c..EW-1 of event 64c+lane (upper-triangle correlation words, cupT
// word-major) against NB individuals whose B rows for this event's slot start
// at LDS byte addresses r[q]: h[q] += popcount(word & B_q word). Blocks of 4
// words: the next block's global loads are issued before this block's gathers.
template <int NB>
__device__ __forceinline__ void corr_chunk(const DevProblem& pb, int c, int lane, const uint32_t (&r)[NB], int (&h)[NB]) {
    const int E = pb.E, EW = pb.EW64, e = 64 * c + lane;
    const bool ev = e < E;
    const uint64_t* src = pb.cupT + (ev ? e : 0);
    uint64_t x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = (ev && c + j < EW) ? src[(size_t)(c + j) * E] : 0ull;
    for (int w = c; w < EW; w += 4) {
        uint64_t y[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = (ev && w + 4 + j < EW) ? src[(size_t)(w + 4 + j) * E] : 0ull;
        uint32_t b[NB];
#pragma unroll
        for (int q = 0; q < NB; ++q) b[q] = r[q] + 8u * (uint32_t)w;
        [&]<int... J>(std::integer_sequence<int, J...>) {
            ([&] {
                if (w + J < EW) {                                  // wave-uniform
                    uint64_t v[NB];
                    lds_gather<NB, 8 * J>(b, v);
#pragma unroll
                    for (int q = 0; q < NB; ++q) h[q] = popc_acc(x[J] & v[q], h[q]);
                }
            }(), ...);
        }(std::make_integer_sequence<int, 4>{});
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = y[j];
    }
}

// corr_chunk, software-pipelined (TT_CORR_SP): the B words of word w+1 for all
// NB individuals are issued (volatile LDS loads: single ds_read_b64, never
// paired into ds_read2_b64, in program order) before word w's popcounts, so
// the compiler's lgkmcnt waits leave the next word's gathers in flight; the
// correlation words stream from HBM/L2 four words ahead. Same-box A/B at syn
// (profiles/r03_s2_ab.json): 5.46 ms against 5.28 for corr_chunk; off.
#ifndef TT_CORR_SP
#define TT_CORR_SP 0
#endif
template <int NB>
__device__ __forceinline__ void corr_chunk_sp(const DevProblem& pb, int c, int lane, const uint32_t (&r)[NB],
                                              int (&h)[NB]) {
    typedef __attribute__((address_space(3))) volatile const uint64_t LdsWord;
    const int E = pb.E, EW = pb.EW64, e = 64 * c + lane;
    const bool ev = e < E;
    const uint64_t* src = pb.cupT + (ev ? e : 0);
    LdsWord* bp[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) bp[q] = (LdsWord*)(size_t)r[q];
    uint64_t x0 = (ev && c < EW) ? src[(size_t)c * E] : 0ull;
    uint64_t x1 = (ev && c + 1 < EW) ? src[(size_t)(c + 1) * E] : 0ull;
    uint64_t x2 = (ev && c + 2 < EW) ? src[(size_t)(c + 2) * E] : 0ull;
    uint64_t x3 = (ev && c + 3 < EW) ? src[(size_t)(c + 3) * E] : 0ull;
    // ping-pong buffers a/b (no register rotation: a copy of an in-flight load
    // would make the compiler wait for it at the copy)
    uint64_t a[NB], b[NB];
#pragma unroll
    for (int q = 0; q < NB; ++q) a[q] = bp[q][c];
    for (int w = c; w < EW; w += 2) {                              // wave-uniform
        if (w + 1 < EW) {
#pragma unroll
            for (int q = 0; q < NB; ++q) b[q] = bp[q][w + 1];
        }
        asm volatile("" ::: "memory");                             // keep the gathers ahead of the popcounts
        const uint64_t x4 = (ev && w + 4 < EW) ? src[(size_t)(w + 4) * E] : 0ull;
#pragma unroll
        for (int q = 0; q < NB; ++q) h[q] = popc_acc(x0 & a[q], h[q]);
        if (w + 1 >= EW) break;
        if (w + 2 < EW) {
#pragma unroll
            for (int q = 0; q < NB; ++q) a[q] = bp[q][w + 2];
        }
        asm volatile("" ::: "memory");
        const uint64_t x5 = (ev && w + 5 < EW) ? src[(size_t)(w + 5) * E] : 0ull;
#pragma unroll
        for (int q = 0; q < NB; ++q) h[q] = popc_acc(x1 & b[q], h[q]);
        x0 = x2; x1 = x3; x2 = x4; x3 = x5;
    }
}

template <int NB, int MEPL>
__global__ __launch_bounds__(1024) void eval_corr_kernel(DevProblem pb, const uint8_t* __restrict__ slot,
                                                         const uint8_t* __restrict__ room, int P,
                                                         int32_t* __restrict__ hcv_out, int32_t* __restrict__ scv_io,
                                                         uint8_t* __restrict__ feas_out, int32_t* __restrict__ pen_out,
                                                         int ablate_arg) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int ablate = TT_EVAL_ABLATE ? ablate_arg : (ablate_arg & 3);   // phase skips: once per tile / batch
    const int E = pb.E, R = pb.R, EW = pb.EW64;
    const CorrLayout L = corr_layout(E, R, EW, NB);
    const int lane = threadIdx.x & 63, wv = wave_id();
    const int NWV = L.NWV, pairs = (EW + 1) / 2, EPL = L.EPL;
    const uint32_t WSI = (uint32_t)L.WSI, BSTB = (uint32_t)L.BST * 8u;
    int32_t* acc = (int32_t*)(lds + L.off_acc);                  // [NB][4]: h, last, bad, -
    int32_t* red = (int32_t*)(lds + L.off_red);                  // [NB][2][64] per-lane h, last partials
    const uint32_t lds0 = lds_addr(lds);

    // build-phase events of this lane and their invariants
    const int eb = (wv * 64 + lane) * EPL;
    // two events per lane from 2-byte aligned rows: one u16 load each
    const bool pair16 = EPL == 2 && (E & 1) == 0 && (((uintptr_t)slot | (uintptr_t)room) & 1) == 0;
    uint64_t possv[MEPL];
    int snv[MEPL];
#pragma unroll
    for (int j = 0; j < MEPL; ++j) {
        const bool ok = j < EPL && eb + j < E;
        possv[j] = ok ? pb.poss[eb + j] : ~0ull;
        snv[j] = ok ? pb.sn[eb + j] : 0;
    }

    const long batches = ((long)P + NB - 1) / NB;
    for (long bt = blockIdx.x; bt < batches; bt += gridDim.x) {
        const long q0 = bt * NB;
        const int nq = (int)min((long)NB, (long)P - q0);
        __syncthreads();                                         // previous batch's outputs are read
        for (int i = threadIdx.x; i < (int)(L.bytes >> 4); i += blockDim.x)
            ((uint4*)lds)[i] = make_uint4(0u, 0u, 0u, 0u);       // workspaces + acc + partials
        __syncthreads();
        // ---- build phase: the lane's events for every individual of the batch
        if (!(ablate & 1)) {
            // every individual's bytes in flight at once (the rows come from HBM)
            uint32_t svq[NB], rvq[NB];
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                svq[q] = 0u; rvq[q] = 0u;
                if (q < nq) {
                    const uint8_t* srow = slot + (q0 + q) * E + eb;
                    const uint8_t* rrow = room + (q0 + q) * E + eb;
                    if (pair16 && eb + 1 < E) {
                        svq[q] = *(const uint16_t*)srow;
                        rvq[q] = *(const uint16_t*)rrow;
                    } else {
#pragma unroll
                        for (int j = 0; j < MEPL; ++j)
                            if (j < EPL && eb + j < E) {
                                svq[q] |= (uint32_t)srow[j] << (8 * j);
                                rvq[q] |= (uint32_t)rrow[j] << (8 * j);
                            }
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                if (q >= nq) break;                              // wave-uniform
                const uint32_t sv = svq[q], rv = rvq[q];
                uint8_t* wsq = lds + (size_t)q * WSI;
                uint64_t* B = (uint64_t*)wsq;
                uint32_t* cnt = (uint32_t*)(wsq + L.off_cnt);
                int h = 0, last = 0;
                bool bad = false;
#pragma unroll
                for (int j = 0; j < MEPL; ++j) {
                    const int e = eb + j;
                    if (j < EPL && e < E) {
                        const uint32_t s = (sv >> (8 * j)) & 0xFFu, ro = (rv >> (8 * j)) & 0xFFu;
                        wsq[L.off_sl + e] = (uint8_t)min(s, (uint32_t)kSlots - 1);   // slot row for the corr phase
                        if (s >= (uint32_t)kSlots || ro >= (uint32_t)R) {
                            bad = true;
                        } else {
                            atomicOr((unsigned long long*)&B[s * (uint32_t)L.BST + (uint32_t)(e >> 6)], 1ull << (e & 63));
                            const uint32_t cell = s * (uint32_t)R + ro, sh = (cell & 1u) << 4;
                            h += (int)((atomicAdd(&cnt[cell >> 1], 1u << sh) >> sh) & 0xFFFFu);
                            h += (int)(((possv[j] >> ro) & 1ull) ^ 1ull);
                            last += ((kLastSlotMask >> s) & 1ull) ? snv[j] : 0;
                        }
                    }
                }
                // per-lane partials (conflict-free, no return); summed once per batch
                atomicAdd(&red[(2 * q) * 64 + lane], h);
                atomicAdd(&red[(2 * q + 1) * 64 + lane], last);
                if (wave_any(bad) && lane == 0) atomicOr(&acc[4 * q + 2], 1);
            }
        }
        __syncthreads();
        // ---- corr phase: the wave's chunk pair against every individual of the batch
        if (!(ablate & 2)) {
            for (int pr = wv; pr < pairs; pr += NWV) {             // wave-uniform
                const int ca = pr, cb = EW - 1 - pr;
                int hq[NB];
#pragma unroll
                for (int q = 0; q < NB; ++q) hq[q] = 0;
#pragma unroll
                for (int side = 0; side < 2; ++side) {
                    const int c = side ? cb : ca;
                    if (side && cb == ca) break;
                    const int e = 64 * c + lane;
                    // per individual: LDS byte address of word 0 of the B row of e's slot
                    uint32_t r[NB];
#pragma unroll
                    for (int q = 0; q < NB; ++q) {
                        const uint32_t sq = (q < nq && e < E) ? (uint32_t)lds[(size_t)q * WSI + L.off_sl + e] : 0u;
                        r[q] = lds0 + (q < nq ? q : 0) * WSI + sq * BSTB;
                    }
#if TT_CORR_SP
                    corr_chunk_sp<NB>(pb, c, lane, r, hq);
#else
                    corr_chunk<NB>(pb, c, lane, r, hq);
#endif
                }
#pragma unroll
                for (int q = 0; q < NB; ++q) {
                    if (q >= nq) break;
                    atomicAdd(&red[(2 * q) * 64 + lane], hq[q]);
                }
            }
        }
        __syncthreads();
        for (int k = wv; k < 2 * nq; k += NWV) {                 // wave-uniform: one sum per row
            const int v = wave_sum(red[k * 64 + lane]);
            if (lane == 0) acc[4 * (k >> 1) + (k & 1)] = v;
        }
        __syncthreads();
        if (threadIdx.x < nq) {
            const long q = q0 + threadIdx.x;
            const int* a = acc + 4 * threadIdx.x;
            if (a[2]) {
                hcv_out[q] = -1; scv_io[q] = -1; feas_out[q] = 0; pen_out[q] = -1;
            } else {
                const int h = a[0], s2 = scv_io[q] + a[1];
                hcv_out[q] = h;
                scv_io[q] = s2;
                feas_out[q] = h == 0 ? 1 : 0;
                pen_out[q] = h == 0 ? s2 : 1000000 + h;
            }
        }
    }
}

// LDS of eval_lanes<16>: the 64-row tile + partials.
static size_t lanes_lds_bytes(int E) {
    int sp = (E + 1 + 3) & ~3;
    if (((sp >> 2) & 1) == 0) sp += 4;
    return (((size_t)64 * sp + 15) & ~(size_t)15) + 4 * (size_t)16 * 64;
}

constexpr size_t kCorrLdsBudget = 152 * 1024;

// Batch size of eval_corr: the largest of 8, 4, 2 whose workspaces fit the LDS
// (0: none).
static int corr_nb(int E, int R, int EW64) {
    for (int nb = 8; nb >= 2; nb >>= 1)
        if (corr_layout(E, R, EW64, nb).bytes <= kCorrLdsBudget) return nb;
    return 0;
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

static bool tile5_fits(const tt_problem* p, int NW) {
    return p->dev.EW64 <= 7 && p->E <= 32767 && tile5_layout(p->E, p->R, NW).bytes <= (NW == 8 ? 80 : 160) * 1024;
}

static bool wide_fits(const tt_problem* p) {
    const int EW64 = p->dev.EW64;
    return p->E <= 32767 && lanes_lds_bytes(p->E) <= 160 * 1024 &&
           corr_nb(p->E, p->R, EW64) > 0 && corr_layout(p->E, p->R, EW64, 2).EPL <= kCorrMaxEPL;
}

// The kernel tt_eval runs for this instance (see tt_eval_variant).
static int auto_variant(const tt_problem* p) {
    if (tile5_fits(p, 8)) return 8;
    if (tile5_fits(p, 4)) return 7;
    if (wide_fits(p)) return 13;
    return 2;
}

extern "C" int tt_eval_auto_variant(const tt_problem* p) { return p ? auto_variant(p) : -1; }

#ifdef TT_T5_STAMP
// profiling build: copies the stamp buffer ([launch][block][10] u64: wave 0's
// start, XCC_ID << 32 | HW_ID, the end of waves 0..7) and, with reset, clears it
extern "C" int tt_t5_stamp_read(unsigned long long* out, int reset) {
    TT_HIP(hipDeviceSynchronize());
    TT_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t5_stamp), sizeof(g_t5_stamp)));
    if (reset) {
        std::vector<unsigned long long> z(sizeof(g_t5_stamp) / 8, 0ull);
        TT_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_t5_stamp), z.data(), sizeof(g_t5_stamp)));
    }
    return kT5Launches * kT5MaxBlocks;
}
#endif

extern "C" int tt_eval_variant(const tt_problem* p, const uint8_t* slot, const uint8_t* room, int P, int32_t* hcv,
                               int32_t* scv, uint8_t* feasible, int32_t* penalty, int variant, void* stream) {
    int rc = check_pop_args(p, P, slot, room);
    if (rc) return rc;
    if (P > 0 && (!hcv || !scv || !feasible || !penalty)) { set_error("null output buffer"); return TT_ERR_INVALID; }
    // profiling-only phase switches (results invalid unless noted): eval_tile5: 1 lane
    // phase, 2 wave phase, 4 correlation words, 8 B-bitset atomics, 16 cell-counter
    // atomics, 32 workspace zeroing, 64 persistent grid, 128 one-tile grid (both valid
    // results); wide path: 1
    // eval_corr build phase, 2 eval_corr corr phase, 4 no eval_corr launch
    const int ablate = variant >> 4;
    variant &= 15;
    if (variant != 0 && variant != 2 && variant != 7 && variant != 8 && variant != 13) {
        set_error("unknown eval variant (0 auto, 2 block, 7/8 tile5, 13 wide)");
        return TT_ERR_INVALID;
    }
    if (P == 0) return TT_OK;
    rc = use_device(p);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int E = p->E, R = p->R;
    if (variant == 0) variant = auto_variant(p);
    if (variant == 13) {
        // wide path: eval_lanes<16> (tile of 64 rows, lane phase) then eval_corr
        if (!wide_fits(p)) { set_error("instance outside the wide eval path"); return TT_ERR_LIMIT; }
        const int EW64 = p->dev.EW64;
        const int tiles = (P + 63) / 64;
        {
            const size_t lds_l = lanes_lds_bytes(E);
            auto launch_l = [&](auto kern) -> int {
                int per_cu = 0;
                TT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 1024, lds_l));
                per_cu = std::min(per_cu, lds_resident_limit(lds_l));    // the 1,280-B LDS block rule
                const int grid = std::min(tiles, std::max(1, per_cu) * p->num_cus);
                hipLaunchKernelGGL(kern, dim3(grid), dim3(1024), lds_l, st, p->dev, slot, P, scv);
                return TT_OK;
            };
            rc = launch_l(eval_lanes_kernel<16>);
            if (rc) return rc;
        }
        if (ablate & 4) return check_hip(hipGetLastError(), "tt_eval launch");   // lane phase only (timing)
        const int NB = corr_nb(E, R, EW64);
        const CorrLayout CL = corr_layout(E, R, EW64, NB);
        auto launch = [&](auto kern) -> int {
            int per_cu = 0;
            TT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * CL.NWV, CL.bytes));
            per_cu = std::min(per_cu, lds_resident_limit(CL.bytes));
            const long batches = ((long)P + NB - 1) / NB;
            const int grid = (int)std::min<long>(batches, (long)std::max(1, per_cu) * p->num_cus);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * CL.NWV), CL.bytes, st, p->dev, slot, room, P, hcv, scv,
                               feasible, penalty, ablate);
            return TT_OK;
        };
        if (CL.EPL <= 2)
            rc = NB == 8 ? launch(eval_corr_kernel<8, 2>) : NB == 4 ? launch(eval_corr_kernel<4, 2>) : launch(eval_corr_kernel<2, 2>);
        else
            rc = NB == 8 ? launch(eval_corr_kernel<8, kCorrMaxEPL>)
                 : NB == 4 ? launch(eval_corr_kernel<4, kCorrMaxEPL>) : launch(eval_corr_kernel<2, kCorrMaxEPL>);
        if (rc) return rc;
    } else if (variant == 7 || variant == 8) {
        // 4 or 8 waves per tile, one tile per workgroup. (16 waves, one workgroup per CU
        // looping over its tiles with the next one staged under the current one: med
        // 82.0 us against 76.0, lg 106.2 against 99.8 -- measured in round 4, removed.)
        const int NW = variant == 7 ? 4 : 8;
        // LDS-DMA staging into two tile buffers when rows are 4-B aligned and the
        // second buffer costs no resident workgroups; else one buffer filled by
        // vector copies. (With one tile per workgroup the second buffer is never
        // filled under compute: only the occupancy decides. At med the 8-wave
        // kernel keeps 2 workgroups per CU either way; the 4-wave kernel fits 4
        // per CU with one buffer, 2 with two.)
        const Tile5Layout L0 = tile5_layout(E, R, NW, false), L1 = tile5_layout(E, R, NW, true);
        const bool db_ok = (E & 3) == 0 && (((uintptr_t)slot) & 3) == 0 && L1.bytes <= 160 * 1024;
        if (p->dev.EW64 > 7 || L0.bytes > 160 * 1024 || E > 32767) {
            set_error("instance too large for the tile5 kernel");
            return TT_ERR_LIMIT;
        }
        const int max_sn = p->max_sn;
        const int pk = (R <= 16 && max_sn <= 0xFFFF) ? 1 : R <= 32 ? 2 : 0;
        const int tiles = (P + 63) / 64;
        // workgroups per CU of the kernel with one or two tile buffers: asked once per
        // problem (the occupancy query costs host time on every launch otherwise)
        auto occupancy = [&](auto kern, size_t bytes, bool two) -> int {
            std::atomic<int>& c = const_cast<tt_problem*>(p)->t5_occ[NW == 8][two];
            int per_cu = c.load(std::memory_order_relaxed);
            if (per_cu >= 0) return per_cu;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * NW, bytes) != hipSuccess) {
                (void)hipGetLastError();    // not sticky: the launch's own error check must not see it
                return 0;
            }
            per_cu = std::min(per_cu, lds_resident_limit(bytes));
            c.store(per_cu, std::memory_order_relaxed);
            return per_cu;
        };
        auto launch = [&](auto kern, size_t bytes, bool two) -> int {
            const int per_cu = occupancy(kern, bytes, two);
            // Grid: with the second tile buffer (two), a persistent grid -- a CU's resident
            // workgroups loop over their tiles with the next one staged by LDS-DMA under
            // the current one. Until round 4 it lost to one tile per workgroup (med -3 %,
            // lg -4 %, P = 262,144 -8 %: the co-resident workgroups ran in lockstep, their
            // stagings together); with the progress-ordered issue priority (TT_T5_PRIO) it
            // wins (profiles/r05_ab_tile5_grid.jsonl: med 71.8 -> 69.7 us, lg 94.3 -> 92.5).
            // Without the second buffer there is nothing to overlap: one tile per workgroup.
            // ablate 64 forces the persistent grid, 128 the one-tile grid (comparisons).
            const bool persist = (ablate & 64) || (TT_T5_PRIO && two && !(ablate & 128));
            const int grid = persist ? std::min(tiles, std::max(1, per_cu) * p->num_cus) : tiles;
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * NW), bytes, st, p->dev, slot, room, P, hcv, scv,
                               feasible, penalty, ablate);
            return TT_OK;
        };
#define TT_T5U(EWC, NWV, PKV)                                                                                      \
    {                                                                                                              \
        const bool db = db_ok && occupancy(eval_tile5_kernel<EWC, NWV, PKV, true>, L1.bytes, true) >=              \
                                     occupancy(eval_tile5_kernel<EWC, NWV, PKV, false>, L0.bytes, false);          \
        rc = db ? launch(eval_tile5_kernel<EWC, NWV, PKV, true>, L1.bytes, true)                                   \
                : launch(eval_tile5_kernel<EWC, NWV, PKV, false>, L0.bytes, false);                                \
    }
#define TT_T5N(EWC, NWV) \
    if (pk == 1) { TT_T5U(EWC, NWV, 1) } else if (pk == 2) { TT_T5U(EWC, NWV, 2) } else { TT_T5U(EWC, NWV, 0) }
#define TT_T5(EWC)                                                      \
    case EWC:                                                           \
        if (NW == 4) { TT_T5N(EWC, 4) } else { TT_T5N(EWC, 8) }         \
        break;
        switch (p->dev.EW64) {
            TT_T5(1) TT_T5(2) TT_T5(3) TT_T5(4) TT_T5(5) TT_T5(6) TT_T5(7)
            default: rc = TT_ERR_LIMIT; break;
        }
#undef TT_T5
#undef TT_T5N
#undef TT_T5U
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

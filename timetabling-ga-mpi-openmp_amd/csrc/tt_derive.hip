// Problem derived data on the device (Problem.cpp:33-58,76-95), the f1 row of
// eventCorrelations = (AᵀA > 0) as an int8 MFMA contraction over the
// students, studentNumber from the diagonal of the same product, and
// possibleRooms from it in the diagonal tiles' epilogue.
//
//   Atb [Ep][Sp/32] u32  event-major BIT image of student_events: bit s of
//                     event e's row is A[s][e]; Ep = E rounded up to 64, Sp = S
//                     rounded up to 128, zero padded (derive_layout, built by the
//                     host from the CSR it needs anyway: one pass over the
//                     nonzeros). 1.3 MB at syn: the operands stay in L2.
//   C = At · Atᵀ      C[i][j] = #students attending both i and j; C[i][i] =
//                     studentNumber[i] since A is 0/1
//
// Mapping: one 4-wave workgroup per 64×64 block (bi <= bj) of C, one 32×32
// quadrant per wave, v_mfma_i32_32x32x32_i8 over 32 students per step with
// exact i32 accumulation. Lane l holds row (l & 31) of its operand tile at
// students 16·(l >> 5) .. +15 of the step: 16 bits of the row's step word,
// expanded in registers to 16 bytes of 0/1 (per nibble x: x·0x00204081 &
// 0x01010101 puts bit k in byte k), for A (events i) and B (events j) alike,
// so the k order is the same on both sides. A lane loads 128 students (four
// steps) of its row with one 16-B load, one chunk ahead (four chunks ahead
// measured 41 us against 37.5 at syn: the waves are bound by the 26 expansion
// VALU per MFMA, not by the L2 loads). C is symmetric,
// so an off-diagonal block's quadrant is written twice: its rows (ballots of
// C > 0 per accumulator register) and its columns (the bits of a lane's own
// accumulators, the two lane halves OR-ed). The image parts written:
//   corr  u32 [E][EW]       eventCorrelations rows (DevProblem::corr)
//   corr64 u64 [E][EW64]    the same rows in 64-bit words
//   cupT  u64 [EW64][E]     upper triangle, word-major (bits j > i)
//   sn    i32 [E]           studentNumber
//   poss  u64 [E]           possibleRooms bitmasks
#include <hip/hip_runtime.h>

#include "tt_internal.h"

namespace ttga {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// 16 bits (students k..k+15 of a row) -> 16 bytes of 0/1, byte j = bit j
__device__ __forceinline__ v4i bits_to_bytes(uint32_t h16) {
    v4i v;
#pragma unroll
    for (int d = 0; d < 4; d++) v[d] = (int)((__builtin_amdgcn_ubfe(h16, 4 * d, 4) * 0x00204081u) & 0x01010101u);
    return v;
}

struct DeriveOut {
    uint32_t* corr;     // [E][EW]
    uint32_t* corr64;   // [E][2·EW64] as u32 words
    uint32_t* cupT;     // [EW64][E] u64 as u32 pairs
    int32_t* sn;        // [E]
    uint64_t* poss;     // [E]
};

__device__ __forceinline__ int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// Writes the 32-bit word of C-row i over columns j0 .. j0+31 to the three images.
__device__ __forceinline__ void put_row_word(const DeriveOut& o, int E, int EW, int EW64, int i, int j0, uint32_t w) {
    if (i >= E) return;
    const int wd = j0 >> 5;
    if (wd < EW) o.corr[(size_t)i * EW + wd] = w;
    o.corr64[(size_t)i * (2 * EW64) + wd] = w;                   // wd < 2·EW64 always (j0 < Ep)
    // upper triangle: bits j > i only
    uint32_t up;
    if (j0 > i) up = w;
    else if (j0 + 31 <= i) up = 0u;
    else up = w & ~((2u << (i - j0)) - 1u);                      // keep bits (i - j0 + 1) .. 31
    o.cupT[((size_t)(j0 >> 6) * E + i) * 2 + (wd & 1)] = up;
}

__global__ __launch_bounds__(256) void derive_corr_kernel(const uint32_t* __restrict__ Atb, int E, int Sp, int nb,
                                                          const int32_t* __restrict__ room_size, int R,
                                                          const uint64_t* __restrict__ efw,
                                                          const uint64_t* __restrict__ rfw, int FW, DeriveOut o) {
    // block pair (bi <= bj) from the linear index, row-major over the upper triangle
    int b = blockIdx.x, bi = 0;
    while (b >= nb - bi) { b -= nb - bi; bi++; }
    const int bj = bi + b;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int qi = w >> 1, qj = w & 1;
    const bool diag_block = bi == bj;
    if (diag_block && qi > qj) return;                         // the transpose of quadrant (0,1)
    const int i0 = 64 * bi + 32 * qi, j0 = 64 * bj + 32 * qj;
    const int r = lane & 31, h = lane >> 5;

    const int SW = Sp >> 5, nch = SW >> 2;                     // u32 words per bit row, 128-student chunks
    const v4i* pa = (const v4i*)(Atb + (size_t)(i0 + r) * SW);
    const v4i* pb = (const v4i*)(Atb + (size_t)(j0 + r) * SW);
    const int sh = 16 * h;
    v16i acc = {};
    v4i na = nch ? pa[0] : v4i{}, nbv = nch ? pb[0] : v4i{};
    for (int c = 0; c < nch; c++) {                            // the next chunk in flight
        const v4i wa = na, wb = nbv;
        if (c + 1 < nch) { na = pa[c + 1]; nbv = pb[c + 1]; }
#pragma unroll
        for (int q = 0; q < 4; q++)
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(bits_to_bytes((uint32_t)wa[q] >> sh),
                                                        bits_to_bytes((uint32_t)wb[q] >> sh), acc, 0, 0, 0);
    }

    const int EW = (E + 31) >> 5, EW64 = (E + 63) >> 6;
    // rows of the quadrant: accumulator register g holds row acc_row(g, h), column r
    uint32_t myrow = 0u;                                       // lane t < 32: the word of row i0 + t
    uint32_t colbits = 0u;                                     // this lane's column r over its 16 rows
#pragma unroll
    for (int g = 0; g < 16; g++) {
        const bool nz = acc[g] > 0;
        const uint64_t bal = ballot(nz);
        // row acc_row(g, 0) is the low half, acc_row(g, 1) the high half
        if (lane == acc_row(g, 0)) myrow = (uint32_t)bal;
        if (lane == acc_row(g, 1)) myrow = (uint32_t)(bal >> 32);
        if (nz) colbits |= 1u << acc_row(g, h);
    }
    const uint32_t col = colbits | (uint32_t)__shfl_xor((int)colbits, 32);
    if (lane < 32) {
        put_row_word(o, E, EW, EW64, i0 + lane, j0, myrow);
        if (!(diag_block && qi == qj)) put_row_word(o, E, EW, EW64, j0 + lane, i0, col);   // C(j, i) rows
    }
    if (diag_block && qi == qj) {
        // studentNumber from the diagonal: (row c, column c) sits in register
        // (c & 3) + 4·(c >> 3) of the lane with column c and half (c >> 2) & 1
        const int c = r;
        if (h == ((c >> 2) & 1)) {
            const int reg = (c & 3) + 4 * (c >> 3);
            int v = 0;
#pragma unroll
            for (int g = 0; g < 16; g++) if (g == reg) v = acc[g];
            const int e = i0 + c;
            if (e < E) {
                o.sn[e] = v;
                // possibleRooms (Problem.cpp:76-95): size fits, every required feature present
                uint64_t pm = 0ull;
                for (int rr = 0; rr < R; rr++) {
                    if (room_size[rr] < v) continue;
                    bool ok = true;
                    for (int f = 0; f < FW; f++) ok &= (efw[(size_t)e * FW + f] & ~rfw[(size_t)rr * FW + f]) == 0ull;
                    if (ok) pm |= 1ull << rr;
                }
                o.poss[e] = pm;
            }
        }
    }
}

}  // namespace

int derive_on_device(const tt_problem* p, const uint32_t* atb, const int32_t* room_size, const uint64_t* efw,
                     const uint64_t* rfw, int FW) {
    const int E = p->E, S = p->S, R = p->R;
    const DeriveLayout DL = derive_layout(E, S);
    const int nb = DL.Ep / 64;
    const size_t at_bytes = ((size_t)DL.Ep * DL.SW * 4 + 255) & ~(size_t)255;
    const size_t rs_bytes = 256 * ((sizeof(int32_t) * R + 255) / 256);
    const size_t ef_bytes = ((sizeof(uint64_t) * E * FW) + 255) & ~(size_t)255;
    const size_t rf_bytes = ((sizeof(uint64_t) * R * FW) + 255) & ~(size_t)255;
    const size_t total = at_bytes + rs_bytes + ef_bytes + rf_bytes + 256;
    uint8_t* tmp = nullptr;
    hipStream_t st = nullptr;
    TT_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipError_t he = hipMalloc(&tmp, total);
    if (he == hipErrorOutOfMemory) {
        // the transient attendance bit image (Ep x Sp / 8 bytes) does not fit: a size
        // limit of this instance, not a device failure
        (void)hipGetLastError();
        (void)hipStreamDestroy(st);
        set_error("tt_problem_create: the " + std::to_string(total >> 20) +
                  " MiB derivation image (E x S attendance bits) does not fit in device memory");
        return TT_ERR_LIMIT;
    }
    if (he != hipSuccess) { (void)hipStreamDestroy(st); return check_hip(he, "derive: hipMalloc"); }
    uint32_t* dAt = (uint32_t*)tmp;
    int32_t* drs = (int32_t*)(tmp + at_bytes);
    uint64_t* def = (uint64_t*)((uint8_t*)drs + rs_bytes);
    uint64_t* drf = (uint64_t*)((uint8_t*)def + ef_bytes);
    const DevProblem& d = p->dev;
    DeriveOut o{const_cast<uint32_t*>(d.corr), (uint32_t*)const_cast<uint64_t*>(d.corr64),
                (uint32_t*)const_cast<uint64_t*>(d.cupT), const_cast<int32_t*>(d.sn), const_cast<uint64_t*>(d.poss)};
    if (DL.SW > 0) he = hipMemcpyAsync(dAt, atb, (size_t)DL.Ep * DL.SW * 4, hipMemcpyHostToDevice, st);
    if (he == hipSuccess) he = hipMemcpyAsync(drs, room_size, sizeof(int32_t) * R, hipMemcpyHostToDevice, st);
    if (he == hipSuccess && FW > 0) he = hipMemcpyAsync(def, efw, sizeof(uint64_t) * E * FW, hipMemcpyHostToDevice, st);
    if (he == hipSuccess && FW > 0) he = hipMemcpyAsync(drf, rfw, sizeof(uint64_t) * R * FW, hipMemcpyHostToDevice, st);
    if (he == hipSuccess)
        hipLaunchKernelGGL(derive_corr_kernel, dim3(nb * (nb + 1) / 2), dim3(256), 0, st, dAt, E, DL.Sp, nb, drs, R, def,
                           drf, FW, o);
    if (he == hipSuccess) he = hipGetLastError();
    if (he == hipSuccess) he = hipStreamSynchronize(st);
    (void)hipFree(tmp);
    (void)hipStreamDestroy(st);
    return check_hip(he, "derive_on_device");
}

}  // namespace ttga

// Problem image: parse-free construction from .tim matrices, derived data
// (Problem.cpp:33-95) and the device upload that replaces the reference's
// MPI_Pack/MPI_Bcast of the Problem (ga.cpp:264-309,417-426).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "tt_internal.h"

namespace ttga {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int check_hip(hipError_t e, const char* what) {
    if (e == hipSuccess) return TT_OK;
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return TT_ERR_DEVICE;
}

int check_pop_args(const tt_problem* p, int P, const void* a, const void* b) {
    if (!p) { set_error("null tt_problem"); return TT_ERR_INVALID; }
    if (P < 0) { set_error("negative population size"); return TT_ERR_INVALID; }
    if (P > 0 && (!a || !b)) { set_error("null population buffer"); return TT_ERR_INVALID; }
    return TT_OK;
}

int use_device(const tt_problem* p) {
    int cur = -1;
    TT_HIP(hipGetDevice(&cur));
    if (cur != p->device) TT_HIP(hipSetDevice(p->device));
    return TT_OK;
}

}  // namespace ttga

using namespace ttga;

extern "C" {

int tt_version(void) { return 1; }

const char* tt_last_error(void) { return g_last_error.c_str(); }

int tt_problem_create(int E, int R, int F, int S, const int32_t* room_size, const int32_t* A,
                      const int32_t* room_feat, const int32_t* event_feat, int device, tt_problem** out) {
    if (!out) { set_error("null output handle"); return TT_ERR_INVALID; }
    *out = nullptr;
    if (E < 1 || E > 65535 || R < 1 || F < 0 || S < 0) { set_error("bad instance dimensions"); return TT_ERR_INVALID; }
    if (R > kMaxRooms) { set_error("more than 64 rooms is not supported"); return TT_ERR_LIMIT; }
    if (!room_size || (S > 0 && !A) || (F > 0 && (!room_feat || !event_feat))) {
        set_error("null instance matrix");
        return TT_ERR_INVALID;
    }
    for (long i = 0; i < (long)R * F; i++)
        if (room_feat[i] != 0 && room_feat[i] != 1) { set_error("room_features must be 0/1"); return TT_ERR_INVALID; }
    for (long i = 0; i < (long)E * F; i++)
        if (event_feat[i] != 0 && event_feat[i] != 1) { set_error("event_features must be 0/1"); return TT_ERR_INVALID; }

    // One pass over student_events: the 0/1 check and the two CSR views (the
    // students' events and the events' students) that the kernels read. The
    // event degrees of the CSR are studentNumber; the device derives it again
    // from the diagonal of AᵀA and the two must agree (checked below).
    std::vector<int32_t> stu_off(S + 1, 0), stu_ev, ev_off(E + 1, 0), ev_stu, degree(E, 0);
    for (int s = 0; s < S; s++) {
        const int32_t* row = A + (size_t)s * E;
        int32_t bad = 0;
        for (int e = 0; e < E; e++) bad |= row[e] & ~1;
        if (bad) { set_error("student_events must be 0/1"); return TT_ERR_INVALID; }
        for (int e = 0; e < E; e++)
            if (row[e]) { stu_ev.push_back(e); degree[e]++; }
        stu_off[s + 1] = (int32_t)stu_ev.size();
    }
    // the attendance matrix as event-major bit rows for the device's AᵀA
    // (csrc/tt_derive.hip derive_layout): bit s of row e = A[s][e], one pass
    // over the nonzeros (1.3 MB at syn instead of a 10-40 MB upload)
    const DeriveLayout DL = derive_layout(E, S);
    std::vector<uint32_t> atb((size_t)DL.Ep * DL.SW, 0u);
    for (int s = 0; s < S; s++)
        for (int k = stu_off[s]; k < stu_off[s + 1]; k++) atb[(size_t)stu_ev[k] * DL.SW + (s >> 5)] |= 1u << (s & 31);

    tt_problem* p = new tt_problem();
    p->E = E; p->R = R; p->F = F; p->S = S; p->device = device;
    const int EW = (E + 31) / 32;
    const int EW64 = (E + 63) / 64;

    for (int e = 0; e < E; e++) ev_off[e + 1] = ev_off[e] + degree[e];
    ev_stu.resize(stu_ev.size());
    {
        std::vector<int32_t> cur(ev_off.begin(), ev_off.end() - 1);
        for (int s = 0; s < S; s++)
            for (int k = stu_off[s]; k < stu_off[s + 1]; k++) ev_stu[cur[stu_ev[k]]++] = s;
    }
    // features as bit words for the device's possibleRooms test
    const int FW = (F + 63) / 64;
    std::vector<uint64_t> efw((size_t)E * FW, 0ull), rfw((size_t)R * FW, 0ull);
    for (int e = 0; e < E; e++)
        for (int f = 0; f < F; f++)
            if (event_feat[(size_t)e * F + f]) efw[(size_t)e * FW + (f >> 6)] |= 1ull << (f & 63);
    for (int r = 0; r < R; r++)
        for (int f = 0; f < F; f++)
            if (room_feat[(size_t)r * F + f]) rfw[(size_t)r * FW + (f >> 6)] |= 1ull << (f & 63);
    std::vector<int32_t> stc_off(S + 1, 0), stc_ev;
    for (int s = 0; s < S; s++) {
        for (int k = stu_off[s]; k < stu_off[s + 1]; k++) stc_ev.push_back(stu_ev[k]);
        while (stc_ev.size() % 8) stc_ev.push_back(E);
        stc_off[s + 1] = (int32_t)stc_ev.size();
    }
    if (stc_ev.empty()) stc_ev.assign(8, E);
    // Student runs for the lane phase: students sorted by their event count
    // rounded up to even (stable), each student's ids padded with E to that
    // count, so a student's list starts on a dword and costs its own size
    // plus at most one sentinel (the 8-id records above pad 22 % of the ids).
    // Wave w of an NW-wave workgroup takes a contiguous range of the sorted
    // students balanced by ids + a per-student constant; its students form
    // runs of one size, (size, first dword, count).
    std::vector<uint16_t> sid;
    std::vector<int32_t> srun_flat;                       // 4 ints per run
    std::vector<int32_t> srun_part(kSrunPartLen, 0);
    if (E <= 32767) {
        std::vector<int> order;
        for (int s = 0; s < S; s++)
            if (stu_off[s + 1] > stu_off[s]) order.push_back(s);
        auto padded = [&](int s) { const int n = stu_off[s + 1] - stu_off[s]; return n + (n & 1); };
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return padded(a) < padded(b); });
        std::vector<int32_t> first(order.size() + 1, 0);  // dword offset of each sorted student
        std::vector<long> cost(order.size() + 1, 0);
        for (size_t i = 0; i < order.size(); i++) {
            const int s = order[i];
            first[i] = (int32_t)(sid.size() / 2);
            for (int k = stu_off[s]; k < stu_off[s + 1]; k++) sid.push_back((uint16_t)stu_ev[k]);
            if (sid.size() & 1) sid.push_back((uint16_t)E);
            cost[i + 1] = cost[i] + padded(s) + 8;
        }
        first[order.size()] = (int32_t)(sid.size() / 2);
        const size_t n_st = order.size();
        for (int nw : {4, 8, 16}) {
            const int base = srun_part_base(nw);
            size_t i = 0;
            for (int w = 0; w < nw; w++) {
                srun_part[base + w] = (int32_t)(srun_flat.size() / 4);
                const long target = cost[n_st] * (w + 1) / nw;
                const size_t i1 = w == nw - 1 ? n_st : std::max(i, (size_t)(std::lower_bound(cost.begin(), cost.end(), target) - cost.begin()));
                for (size_t j = i; j < i1;) {
                    const int ne = padded(order[j]);
                    size_t k = j;
                    while (k < i1 && padded(order[k]) == ne) k++;
                    srun_flat.insert(srun_flat.end(), {ne, first[j], (int32_t)(k - j), 0});
                    j = k;
                }
                i = i1;
            }
            srun_part[base + nw] = (int32_t)(srun_flat.size() / 4);
        }
    }
    sid.resize(sid.size() + 32, (uint16_t)E);             // slack for 64-B scalar over-reads
    if (srun_flat.empty()) srun_flat.assign(4, 0);
    p->nnz_students = (int)stu_ev.size();

    // One device block, 256-B aligned sub-buffers.
    struct Part { const void* src; size_t bytes; size_t off; };
    std::vector<Part> parts = {
        {nullptr, sizeof(int32_t) * E, 0},                      // studentNumber (device-derived)
        {stu_off.data(), sizeof(int32_t) * (S + 1), 0},
        {stu_ev.data(), sizeof(int32_t) * stu_ev.size(), 0},
        {ev_off.data(), sizeof(int32_t) * (E + 1), 0},
        {ev_stu.data(), sizeof(int32_t) * ev_stu.size(), 0},
        {nullptr, sizeof(uint64_t) * E, 0},                     // possibleRooms (device-derived)
        {nullptr, sizeof(uint32_t) * E * EW, 0},                // eventCorrelations (device-derived)
        {nullptr, sizeof(int32_t) * 4, 0},   // status word
        {nullptr, sizeof(uint64_t) * EW64 * E, 0},              // cupT (device-derived)
        {stc_off.data(), sizeof(int32_t) * stc_off.size(), 0},
        {stc_ev.data(), sizeof(int32_t) * stc_ev.size(), 0},
        {nullptr, sizeof(uint64_t) * E * EW64, 0},              // corr64 (device-derived)
        {sid.data(), sizeof(uint16_t) * sid.size(), 0},
        {srun_flat.data(), sizeof(int32_t) * srun_flat.size(), 0},
        {srun_part.data(), sizeof(int32_t) * srun_part.size(), 0},
    };
    size_t total = 0;
    for (auto& q : parts) { q.off = total; total += (q.bytes + 255) & ~(size_t)255; }
    total = std::max<size_t>(total, 256);

    int prev = 0;
    hipError_t he = hipGetDevice(&prev);
    if (he == hipSuccess) he = hipSetDevice(device);
    if (he == hipSuccess) he = hipDeviceGetAttribute(&p->num_cus, hipDeviceAttributeMultiprocessorCount, device);
    if (he == hipSuccess) he = hipMalloc(&p->dev_block, total);
    if (he != hipSuccess) { check_hip(he, "tt_problem_create"); delete p; return TT_ERR_DEVICE; }
    std::vector<uint8_t> staging(total, 0);
    for (auto& q : parts)
        if (q.src && q.bytes) memcpy(staging.data() + q.off, q.src, q.bytes);
    he = hipMemcpy(p->dev_block, staging.data(), total, hipMemcpyHostToDevice);
    if (he != hipSuccess) { check_hip(he, "tt_problem_create upload"); (void)hipFree(p->dev_block); delete p; return TT_ERR_DEVICE; }

    uint8_t* base = (uint8_t*)p->dev_block;
    DevProblem& d = p->dev;
    d.E = E; d.R = R; d.S = S; d.EW = EW;
    d.sn = (const int32_t*)(base + parts[0].off);
    d.stu_off = (const int32_t*)(base + parts[1].off);
    d.stu_ev = (const int32_t*)(base + parts[2].off);
    d.ev_off = (const int32_t*)(base + parts[3].off);
    d.ev_stu = (const int32_t*)(base + parts[4].off);
    d.poss = (const uint64_t*)(base + parts[5].off);
    d.corr = (const uint32_t*)(base + parts[6].off);
    d.status = (int32_t*)(base + parts[7].off);
    d.EW64 = EW64;
    d.cupT = (const uint64_t*)(base + parts[8].off);
    d.stc_off = (const int32_t*)(base + parts[9].off);
    d.stc_ev = (const int32_t*)(base + parts[10].off);
    d.corr64 = (const uint64_t*)(base + parts[11].off);
    d.sid = (const uint32_t*)(base + parts[12].off);
    d.srun = (const int4*)(base + parts[13].off);
    d.srun_part = (const int32_t*)(base + parts[14].off);

    // studentNumber, eventCorrelations (and its two other layouts) and
    // possibleRooms: the MFMA derivation (csrc/tt_derive.hip)
    int rc = TT_OK;
    he = hipSetDevice(device);
    if (he != hipSuccess) rc = check_hip(he, "tt_problem_create");
    if (rc == TT_OK) rc = derive_on_device(p, atb.data(), room_size, efw.data(), rfw.data(), FW);
    // host copies for tt_problem_derived and the kernels' launch choices
    p->student_number.assign(E, 0);
    p->poss_bits.assign(E, 0ull);
    p->corr_bits.assign((size_t)E * EW, 0u);
    if (rc == TT_OK) rc = check_hip(hipMemcpy(p->student_number.data(), d.sn, sizeof(int32_t) * E, hipMemcpyDeviceToHost), "tt_problem_create readback");
    if (rc == TT_OK) rc = check_hip(hipMemcpy(p->poss_bits.data(), d.poss, sizeof(uint64_t) * E, hipMemcpyDeviceToHost), "tt_problem_create readback");
    if (rc == TT_OK) rc = check_hip(hipMemcpy(p->corr_bits.data(), d.corr, sizeof(uint32_t) * E * EW, hipMemcpyDeviceToHost), "tt_problem_create readback");
    if (rc == TT_OK && !p->student_number.empty())
        p->max_sn = *std::max_element(p->student_number.begin(), p->student_number.end());
    if (rc == TT_OK && p->student_number != degree) {
        set_error("tt_problem_create: device studentNumber differs from the attendance counts");
        rc = TT_ERR_DEVICE;
    }
    (void)hipSetDevice(prev);
    if (rc != TT_OK) {
        (void)hipFree(p->dev_block);
        delete p;
        return rc;
    }
    *out = p;
    return TT_OK;
}

int tt_problem_destroy(tt_problem* p) {
    if (!p) return TT_OK;
    int rc = TT_OK;
    if (p->dev_block) {
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(p->device);
        if (!p->ls_redo.empty()) {                      // redo lists may be in use on their streams
            (void)hipDeviceSynchronize();
            for (auto& r : p->ls_redo) {
                (void)hipFreeAsync(r.list, nullptr);
                if (r.ph_dev) (void)hipFreeAsync(r.ph_dev, nullptr);
            }
            (void)hipDeviceSynchronize();
            for (auto& r : p->ls_redo) {
                if (r.ph_host) (void)hipHostFree((void*)r.ph_host);
                for (hipEvent_t e : r.ev)
                    if (e) (void)hipEventDestroy(e);
            }
        }
        rc = check_hip(hipFree(p->dev_block), "tt_problem_destroy");
        (void)hipSetDevice(prev);
    }
    delete p;
    return rc;
}

int tt_problem_dims(const tt_problem* p, int32_t* dims) {
    if (!p || !dims) { set_error("null argument"); return TT_ERR_INVALID; }
    dims[0] = p->E; dims[1] = p->R; dims[2] = p->F; dims[3] = p->S;
    return TT_OK;
}

int tt_problem_derived(const tt_problem* p, int32_t* student_number, int32_t* corr, int32_t* possible) {
    if (!p) { set_error("null tt_problem"); return TT_ERR_INVALID; }
    const int E = p->E, R = p->R, EW = (E + 31) / 32;
    if (student_number) std::copy(p->student_number.begin(), p->student_number.end(), student_number);
    if (corr)
        for (int i = 0; i < E; i++)
            for (int j = 0; j < E; j++) corr[(size_t)i * E + j] = (p->corr_bits[(size_t)i * EW + (j >> 5)] >> (j & 31)) & 1u;
    if (possible)
        for (int i = 0; i < E; i++)
            for (int j = 0; j < R; j++) possible[(size_t)i * R + j] = (int32_t)((p->poss_bits[i] >> j) & 1ull);
    return TT_OK;
}

int tt_device_status(const tt_problem* p, int32_t* status) {
    if (!p || !status) { set_error("null argument"); return TT_ERR_INVALID; }
    int rc = use_device(p);
    if (rc) return rc;
    TT_HIP(hipDeviceSynchronize());
    TT_HIP(hipMemcpy(status, p->dev.status, sizeof(int32_t), hipMemcpyDeviceToHost));
    return TT_OK;
}

}  // extern "C"

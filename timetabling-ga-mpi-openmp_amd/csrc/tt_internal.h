// Host-side internals shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ttga.h"
#include "tt_common.h"

struct tt_problem {
    int E, R, F, S, device, num_cus;
    // host copies (tt_problem_derived, validation)
    std::vector<int32_t> student_number;
    std::vector<uint64_t> poss_bits;
    std::vector<uint32_t> corr_bits;
    int nnz_students;
    // device allocations
    void* dev_block;
    ttga::DevProblem dev;
    // local search redo lists, one per stream (count, done counter, entries):
    // zeroed once when allocated, reset on the device by the redo launch;
    // ls_mu is held while a call enqueues its launches, so two host threads on
    // one stream cannot interleave their first and redo launches
    struct LsRedo {
        void* stream;
        int32_t* list;
        int cap;
        // phase-2 steps and all steps of the stream's local-search calls: counted
        // on the device (ph_dev), copied after call k into pinned host memory
        // ph_host[2 (k & 1) ..] with event ev[k & 1] recorded behind the copy;
        // call k + 2 waits for that event and decides the phase-2 student masks'
        // launch from those counts (tt_ls.hip), so a launch's shape depends only
        // on the sequence of calls, never on host/device timing
        unsigned long long* ph_dev = nullptr;
        volatile unsigned long long* ph_host = nullptr;
        hipEvent_t ev[2] = {nullptr, nullptr};
        long calls = 0;
        int sms_last = 0;        // students with masks in the last call's first launch
    };
    std::vector<LsRedo> ls_redo;
    std::mutex ls_mu;
    // students with phase-2 masks in the local search, per matcher-task cap
    // (full, small); -1 until the first call decides (tt_ls.hip ls_mask_students)
    std::atomic<int> ls_smask[2] = {-1, -1};
    // eval_tile5 launch decisions, per wave count (4, 8) and tile buffers (1, 2):
    // workgroups per CU, -1 until the first launch asks (tt_eval.hip); and the
    // largest studentNumber (packing choice), set at creation
    std::atomic<int> t5_occ[2][2] = {{-1, -1}, {-1, -1}};
    int max_sn = 0;
};

namespace ttga {

void set_error(const std::string& msg);

// Returns TT_OK or records the HIP error and returns TT_ERR_DEVICE.
int check_hip(hipError_t e, const char* what);

#define TT_HIP(call)                                         \
    do {                                                     \
        int _rc = ::ttga::check_hip((call), #call);          \
        if (_rc != TT_OK) return _rc;                        \
    } while (0)

// Workgroups of `lds_bytes` of LDS each that one gfx950 CU actually keeps
// resident: LDS is allocated in blocks of 1,280 B (160 KB / 128), which
// hipOccupancyMaxActiveBlocksPerMultiprocessor does not model (it divides
// 160 KB by the size rounded to 256 B: 20 against the real 18 at 8,032 B).
// Measured by tools/occ_probe.hip (profiles/r05_occ_sweep.jsonl).
inline int lds_resident_limit(size_t lds_bytes) {
    const size_t blocks = (lds_bytes + 1279) / 1280;
    return blocks == 0 ? 1 << 30 : (int)(128 / blocks);
}

// Common argument checks for population entry points.
int check_pop_args(const tt_problem* p, int P, const void* a, const void* b);

// Makes the handle's device current for the calling thread.
int use_device(const tt_problem* p);

// Bit image of the attendance matrix for the device derivation: Ep = E rounded
// up to 64 event rows of SW u32 words, Sp = S rounded up to 128 students (one
// 16-B load per lane per chunk).
struct DeriveLayout {
    int Ep, Sp, SW;
};
inline DeriveLayout derive_layout(int E, int S) {
    DeriveLayout L;
    L.Ep = (E + 63) & ~63;
    L.Sp = (S + 127) & ~127;
    L.SW = L.Sp / 32;
    return L;
}

// studentNumber, eventCorrelations (corr, corr64, cupT) and possibleRooms of
// the image, derived on the handle's (current) device from the attendance bit
// rows atb[Ep][SW] (derive_layout; csrc/tt_derive.hip); synchronous.
int derive_on_device(const tt_problem* p, const uint32_t* atb, const int32_t* room_size, const uint64_t* efw,
                     const uint64_t* rfw, int FW);

}  // namespace ttga

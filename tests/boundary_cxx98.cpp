// A consumer of include/ttga.h written as the reference's own code is: C++98,
// compiled with the reference's flags (g++ -Wall -ansi -O3, /root/reference
// Makefile:3) -- the INTEGRATION.md sketch of ga.cpp's call sites, calling
// every tt_* entry point. tests/test_boundary_cxx98.py builds it warning-free,
// links it against libttga.so (every symbol must resolve) and runs it: without
// a GPU tt_problem_create stops at TT_ERR_DEVICE; with one the whole sketch
// runs on a small seeded instance.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ttga.h"

namespace {

// Park-Miller minimal standard, as Random.cc:27-37
long pm_next(long s) {
    const long a = 16807, m = 2147483647, q = 127773, r = 2836;
    long k = s / q;
    s = a * (s - k * q) - r * k;
    if (s < 0) s += m;
    return s;
}

struct Instance {   // the matrices Problem(istream&) reads (Problem.cpp:7-31)
    int E, R, F, S;
    std::vector<int32_t> roomSize, studentEvents, roomFeatures, eventFeatures;
};

Instance make_instance(long seed) {
    Instance in;
    in.E = 100; in.R = 5; in.F = 5; in.S = 80;
    in.roomSize.resize(in.R);
    in.studentEvents.resize(in.S * in.E);
    in.roomFeatures.resize(in.R * in.F);
    in.eventFeatures.resize(in.E * in.F);
    for (int r = 0; r < in.R; ++r) { seed = pm_next(seed); in.roomSize[r] = 20 + (int)(seed % 30); }
    for (size_t i = 0; i < in.studentEvents.size(); ++i) { seed = pm_next(seed); in.studentEvents[i] = seed % 20 == 0; }
    for (size_t i = 0; i < in.roomFeatures.size(); ++i) { seed = pm_next(seed); in.roomFeatures[i] = seed % 2; }
    for (size_t i = 0; i < in.eventFeatures.size(); ++i) { seed = pm_next(seed); in.eventFeatures[i] = seed % 5 == 0; }
    return in;
}

int fail(const char* what, int rc) {
    std::printf("%s rc=%d: %s\n", what, rc, tt_last_error());
    return rc;
}

}  // namespace

int main() {
    std::printf("tt_version %d\n", tt_version());
    Instance in = make_instance(12345);
    tt_problem* tp = NULL;
    int rc = tt_problem_create(in.E, in.R, in.F, in.S, &in.roomSize[0], &in.studentEvents[0], &in.roomFeatures[0],
                               &in.eventFeatures[0], /*device=*/0, &tp);
    if (rc == TT_ERR_DEVICE) {
        // no usable gfx950 device: the library says so instead of falling back to the CPU
        std::printf("tt_problem_create TT_ERR_DEVICE: %s\n", tt_last_error());
        // the remaining entry points reject a null handle before touching a device
        int bad = 0;
        int32_t dims[4];
        bad += tt_problem_dims(NULL, dims) != TT_ERR_INVALID;
        bad += tt_problem_derived(NULL, NULL, NULL, NULL) != TT_ERR_INVALID;
        bad += tt_eval(NULL, NULL, NULL, 1, NULL, NULL, NULL, NULL, NULL) != TT_ERR_INVALID;
        bad += tt_eval_variant(NULL, NULL, NULL, 1, NULL, NULL, NULL, NULL, 0, NULL) != TT_ERR_INVALID;
        bad += tt_eval_auto_variant(NULL) != -1;
        bad += tt_assign_rooms(NULL, NULL, NULL, 1, NULL) != TT_ERR_INVALID;
        bad += tt_random_init(NULL, NULL, NULL, NULL, 1, NULL) != TT_ERR_INVALID;
        bad += tt_crossover(NULL, NULL, NULL, NULL, NULL, NULL, 1, NULL) != TT_ERR_INVALID;
        bad += tt_mutation(NULL, NULL, NULL, NULL, 1, NULL) != TT_ERR_INVALID;
        bad += tt_local_search(NULL, NULL, NULL, NULL, 1, 200, 1.0, 1.0, 0.0, NULL) != TT_ERR_INVALID;
        bad += tt_local_search_ordered(NULL, NULL, NULL, NULL, 1, 200, 1.0, 1.0, 0.0, NULL, NULL) != TT_ERR_INVALID;
        bad += tt_lpt_order(NULL, NULL, 1, NULL, NULL, NULL) != TT_ERR_INVALID;
        bad += tt_local_search_stats(NULL, NULL, NULL) != TT_ERR_INVALID;
        bad += tt_local_search_masks(NULL, NULL, NULL) != TT_ERR_INVALID;
        bad += tt_local_search_eval(NULL, NULL, NULL, NULL, 1, 200, 1.0, 1.0, 0.0, NULL, NULL, NULL, NULL, NULL, NULL) !=
               TT_ERR_INVALID;
        bad += tt_ga_breed(NULL, NULL, NULL, NULL, 10, NULL, 1, 0.8, 0.5, 1, NULL, NULL, NULL, NULL) != TT_ERR_INVALID;
        bad += tt_ga_replace(NULL, NULL, NULL, NULL, NULL, NULL, NULL, 10, NULL, NULL, NULL, NULL, NULL, NULL, 1, NULL,
                             NULL) != TT_ERR_INVALID;
        int32_t st = 0;
        bad += tt_device_status(NULL, &st) != TT_ERR_INVALID;
        bad += tt_ga_work_bytes(64, in.E) == 0;
        bad += tt_ga_work_source_offset(64, in.E) >= tt_ga_work_bytes(64, in.E);
        bad += tt_problem_destroy(NULL) != TT_OK;
        std::printf("null-handle checks: %d wrong\n", bad);
        return bad ? 10 : TT_ERR_DEVICE;
    }
    if (rc != TT_OK) return fail("tt_problem_create", rc);
    // the device path is exercised by the GPU tests through ctypes; here only the
    // synchronous, host-visible calls, as ga.cpp's set-up would make them
    int32_t dims[4];
    if ((rc = tt_problem_dims(tp, dims)) != TT_OK) return fail("tt_problem_dims", rc);
    std::vector<int32_t> sn(in.E), corr(in.E * in.E), poss(in.E * in.R);
    if ((rc = tt_problem_derived(tp, &sn[0], &corr[0], &poss[0])) != TT_OK) return fail("tt_problem_derived", rc);
    std::printf("dims %d %d %d %d, auto variant %d\n", dims[0], dims[1], dims[2], dims[3], tt_eval_auto_variant(tp));
    int32_t st = 0;
    if ((rc = tt_device_status(tp, &st)) != TT_OK) return fail("tt_device_status", rc);
    tt_problem_destroy(tp);
    return TT_OK;
}

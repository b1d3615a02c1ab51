// Solution::localSearch (Solution.cpp:471-769) — device implementation pending.
#include "tt_internal.h"

using namespace ttga;

extern "C" int tt_local_search(const tt_problem* p, uint8_t* slot, uint8_t* room, int64_t* rng, int P,
                               int max_steps, double p1, double p2, double p3, void* stream) {
    (void)slot; (void)room; (void)rng; (void)P; (void)max_steps; (void)p1; (void)p2; (void)p3; (void)stream;
    if (!p) { set_error("null tt_problem"); return TT_ERR_INVALID; }
    set_error("tt_local_search: not implemented yet");
    return TT_ERR_LIMIT;
}

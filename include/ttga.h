/* ttga.h — C-ABI of the MI355X-native evaluation-and-evolution engine for the
 * Rossi-Doria/Paechter course-timetabling GA (drop-in for the hot path of
 * nelilepo/timetabling-ga-mpi-openmp).
 *
 * The reference has no FFI layer: its boundary is the C++ class API of
 * Problem (Problem.h:32-51) and Solution (Solution.h:33-83), called only from
 * ga.cpp. Each entry point below replaces one of those calls, batched over a
 * population of P individuals that lives in device memory (HBM):
 *
 *   population layout (caller-owned device buffers, individual-major):
 *     slot[P][E]  uint8  timeslot of each event, 0..44   (Solution::sln[e].first)
 *     room[P][E]  uint8  room of each event, 0..R-1      (Solution::sln[e].second)
 *     rng[P]      int64  one Park-Miller state per individual (Random::seed)
 *
 * Conventions: every function returns TT_OK (0) or a TT_ERR_* code and never
 * throws; tt_last_error() gives a message for the calling thread. Every
 * device-side call is asynchronous on the caller's stream (a hipStream_t
 * passed as void*; NULL = default stream). One tt_problem may be used by
 * several host threads on different streams. Nothing here falls back to the
 * CPU: without a usable gfx950 device the calls fail with TT_ERR_DEVICE.
 *
 * Limits: 1 <= E <= 65535, 1 <= R <= 64, S >= 0, F >= 0; at most 256 events
 * share one timeslot inside tt_assign_rooms/tt_local_search (beyond that the
 * affected rooms are written as 255 and tt_device_status() reports it).
 */
#ifndef TTGA_H
#define TTGA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TT_OK 0
#define TT_ERR_INVALID 1   /* bad argument (null pointer, size, non-binary matrix) */
#define TT_ERR_DEVICE 2    /* HIP runtime/device failure */
#define TT_ERR_LIMIT 3     /* instance outside the documented limits */

#define TT_NUM_SLOTS 45    /* 5 days x 9 slots, Solution.cpp:52,57 */

typedef struct tt_problem tt_problem;

/* Replaces Problem::Problem(istream&) (Problem.cpp:3-96) and the MPI problem
 * broadcast (ga.cpp:417-426): takes the parsed .tim matrices, derives
 * studentNumber (Problem.cpp:33-40), eventCorrelations (:42-58) and
 * possibleRooms (:76-95) exactly as the reference, and uploads the device
 * image to `device`. The derivation runs on the device: eventCorrelations =
 * (A^T A > 0) as an int8 MFMA contraction over the students, studentNumber
 * from its diagonal, possibleRooms in the same launch (csrc/tt_derive.hip);
 * the host builds only the sparse (CSR) views of A. Synchronous.
 *   room_size[R], student_events[S*E] (row-major, 0/1), room_features[R*F],
 *   event_features[E*F] (0/1). */
int tt_problem_create(int E, int R, int F, int S, const int32_t* room_size, const int32_t* student_events,
                      const int32_t* room_features, const int32_t* event_features, int device,
                      tt_problem** out);

/* Problem::~Problem (Problem.cpp:114-120). */
int tt_problem_destroy(tt_problem* p);

/* dims[0..3] = E, R, F, S (Problem.h:35-38). */
int tt_problem_dims(const tt_problem* p, int32_t* dims);

/* Host copies of the derived matrices (Problem.h:39,42,46); any pointer may be NULL.
 *   student_number[E], corr[E*E], possible[E*R]. */
int tt_problem_derived(const tt_problem* p, int32_t* student_number, int32_t* corr, int32_t* possible);

/* Batched Solution::computeFeasibility / computeHcv / computeScv /
 * computePenalty (Solution.cpp:63-170; penalty = scv if feasible else
 * 1000000 + hcv). Outputs are device buffers of length P. hcv and scv are
 * always both computed. An individual with slot >= 45 or room >= R is
 * reported as hcv = scv = penalty = -1, feasible = 0. */
int tt_eval(const tt_problem* p, const uint8_t* slot, const uint8_t* room, int P, int32_t* hcv, int32_t* scv,
            uint8_t* feasible, int32_t* penalty, void* stream);

/* tt_eval with an explicit kernel choice, for tests and profiling:
 *   0 = automatic (8 when its LDS fits, else 7, else 13, else 2),
 *   2 = eval_block, one workgroup per individual (any E),
 *   7/8 = eval_tile5, 4/8 waves per 64-individual tile (E <= 448): a
 *         lane-per-individual phase (attendance masks) and a wave-per-individual
 *         phase (bitset hard constraints), slot rows staged by LDS-DMA,
 *   13 = wide path: eval_lanes (16-wave lane-phase tile) + eval_corr (batches
 *        of individuals against the streamed correlation triangle; E <= 2490,
 *        the 64-row tile must fit the LDS; automatic for E > 448).
 * Bits 4 and up of `variant` are profiling switches (csrc/tt_eval.hip); most
 * of them give invalid results. All variants give identical results. */
int tt_eval_variant(const tt_problem* p, const uint8_t* slot, const uint8_t* room, int P, int32_t* hcv,
                    int32_t* scv, uint8_t* feasible, int32_t* penalty, int variant, void* stream);

/* The variant tt_eval chooses for this instance: 8 or 7 (E <= 448), 13 (the
 * wide path, E <= 2490), else 2 (eval_block); -1 for a null handle. */
int tt_eval_auto_variant(const tt_problem* p);

/* Solution::assignRooms (Solution.cpp:772-891) on every non-empty timeslot in
 * ascending order, events of a slot in ascending index: the max-cardinality
 * matching found by the reference's priority-first-search augmentation,
 * unmatched events sent to the least-busy possible room (busy[] starting at
 * 0). Writes room[P][E]. */
int tt_assign_rooms(const tt_problem* p, const uint8_t* slot, uint8_t* room, int P, void* stream);

/* Solution::RandomInitialSolution (Solution.cpp:48-61) per individual, each
 * with its own Random stream rng[i] (advanced in place by E draws). */
int tt_random_init(const tt_problem* p, int64_t* rng, uint8_t* slot, uint8_t* room, int P, void* stream);

/* Solution::crossover (Solution.cpp:893-910) into a fresh child: per event,
 * next() < 0.5 takes parent 1's slot else parent 2's, then assignRooms.
 * parent1/parent2/child are [P][E] slot arrays; rng advanced by E draws. */
int tt_crossover(const tt_problem* p, const uint8_t* slot1, const uint8_t* slot2, int64_t* rng, uint8_t* slot,
                 uint8_t* room, int P, void* stream);

/* Solution::mutation -> randomMove (Solution.cpp:441-469,912-914), in place. */
int tt_mutation(const tt_problem* p, uint8_t* slot, uint8_t* room, int64_t* rng, int P, void* stream);

/* Solution::localSearch(maxSteps, LS_limit, p1, p2, p3) (Solution.cpp:471-769)
 * per individual with its own Random stream; in place. The LS_limit wall-clock
 * bound (999999 s by default, never binding) is not modelled. */
int tt_local_search(const tt_problem* p, uint8_t* slot, uint8_t* room, int64_t* rng, int P, int max_steps,
                    double p1, double p2, double p3, void* stream);

/* tt_local_search with the individuals dispatched in the order order[0..P-1]
 * (device i32, a permutation of 0..P-1; NULL: 0..P-1). Every individual's
 * result is the same as tt_local_search's; only the wave launch order changes
 * (longest-expected first shortens the launch's tail). An order that is not a
 * permutation sets tt_device_status bit 3. */
int tt_local_search_ordered(const tt_problem* p, uint8_t* slot, uint8_t* room, int64_t* rng, int P, int max_steps,
                            double p1, double p2, double p3, const int32_t* order, void* stream);

/* tt_local_search_ordered followed by the evaluation of every searched
 * individual (localSearch, then computePenalty: ga.cpp:574-575), in the same
 * launch: hcv, scv, penalty (i32) and feasible (u8) of individual i, as tt_eval
 * would give them for the searched row (the -1 sentinels for an invalid genome,
 * which the search leaves untouched). The four outputs are all given or all
 * NULL (NULL: tt_local_search_ordered). */
int tt_local_search_eval(const tt_problem* p, uint8_t* slot, uint8_t* room, int64_t* rng, int P, int max_steps,
                         double p1, double p2, double p3, const int32_t* order, int32_t* hcv, int32_t* scv,
                         uint8_t* feasible, int32_t* penalty, void* stream);

/* Diagnostics: the step counts of the last tt_local_search call on `stream`
 * (waits for that call's counts, not for the whole stream): steps[0] = steps
 * taken in phase 2, steps[1] = all steps (0, 0 before any call on the stream
 * of an instance with more than 64 events). Call k on a stream launches the
 * phase-2 student masks by the phase-2 share of call k - 2 (waiting for that
 * call's counts if they have not landed), so a launch's shape depends only on
 * the sequence of calls; results never depend on it. */
int tt_local_search_stats(const tt_problem* p, void* stream, uint64_t* steps);

/* Diagnostics: students with phase-2 masks in the first launch of the last
 * tt_local_search call on `stream` (0: no masks; -1: no such call yet). */
int tt_local_search_masks(const tt_problem* p, void* stream, int32_t* students);

/* A longest-expected-first dispatch order for tt_local_search_ordered:
 * order[0..n-1] = the indices of key[0..n-1] (device i32, e.g. the children's
 * hcv before their local search) by key descending, ties by index, negative
 * keys last. work: device scratch of at least 8 * (n rounded up to a power of
 * two) bytes (tt_ga_work_bytes(n, E) suffices). */
int tt_lpt_order(const tt_problem* p, const int32_t* key, int n, int32_t* order, void* work, void* stream);

/* ---- GA generation primitives (ga.cpp:510-588, batched over C children) ----
 * Population (caller-owned, device): pop_slot/pop_room [N][E], pop_hcv,
 * pop_scv, pop_penalty i32[N], pop_feasible u8[N]; kept sorted by penalty.
 *
 * tt_ga_breed: for every child c, on its own stream rng[c], in the reference's
 * per-generation draw order (ga.cpp:543-571): optionally the 3*E draws of the
 * three discarded RandomInitialSolution calls (ga.cpp:543-548), two
 * selection5 tournaments over pop_penalty (ga.cpp:129-145), next() < p_cross ?
 * crossover of the two parents : copy of the first (ga.cpp:562-566), then
 * next() < p_mut ? randomMove (ga.cpp:569-571). Children come out with rooms
 * assigned, ready for tt_local_search + tt_eval. child_flags u8[C] (scratch:
 * bit 0 crossed, bit 1 mutated). */
int tt_ga_breed(const tt_problem* p, const uint8_t* pop_slot, const uint8_t* pop_room, const int32_t* pop_penalty,
                int N, int64_t* rng, int C, double p_cross, double p_mut, int skip_init_draws, uint8_t* child_slot,
                uint8_t* child_room, uint8_t* child_flags, void* stream);

/* Bytes of device scratch tt_ga_replace needs for a population of N (also
 * enough for tt_lpt_order over n <= N keys). */
size_t tt_ga_work_bytes(int N, int E);

/* Byte offset, inside a tt_ga_work_bytes(N, E) work buffer, of the int32 that
 * tt_ga_replace leaves there: the merged position the new pop[0] came from
 * (N-C+c for child c, else its old position), which the drivers report as
 * the logEntry threadID (ga.cpp:498,580-585). Only tt_ga_replace writes it;
 * tt_lpt_order and the rest of the scratch never touch it. */
size_t tt_ga_work_source_offset(int N, int E);

/* tt_ga_replace: the C evaluated children overwrite population positions
 * N-C..N-1 (ga.cpp:582, "pop[popSize-1]->copy(child)" for C = 1), then the
 * population is sorted by penalty ascending (ga.cpp:583; ties keep position
 * order, std::sort leaves them unspecified). Penalties compare as unsigned,
 * so an invalid genome (penalty -1) sorts last; tt_ga_breed's selection5
 * ranks it last the same way. In place; `work` has tt_ga_work_bytes(N, E)
 * bytes. On return the int32 at tt_ga_work_source_offset(N, E) holds the
 * merged position the new pop[0] came from (N-C+c for child c). */
int tt_ga_replace(const tt_problem* p, uint8_t* pop_slot, uint8_t* pop_room, int32_t* pop_hcv, int32_t* pop_scv,
                  uint8_t* pop_feasible, int32_t* pop_penalty, int N, const uint8_t* child_slot,
                  const uint8_t* child_room, const int32_t* child_hcv, const int32_t* child_scv,
                  const uint8_t* child_feasible, const int32_t* child_penalty, int C, void* work, void* stream);

/* Device-side status word of the problem handle (sticky, OR of):
 *   bit 0 (1)  a slot exceeded 256 events in a matching; its rooms were written as 255;
 *   bit 1 (2)  tt_local_search met an invalid genome (slot >= 45 or room >= R) and
 *              left that individual untouched;
 *   bit 2 (4)  tt_local_search's loop bound fired. Unreachable: a visit either
 *              counts towards evCount < E or accepts a move, which costs a step,
 *              so a phase makes at most (maxSteps + 2) * E visits
 *              (Solution.cpp:498-505,616-618) and the bound is twice that per
 *              phase; tests assert it never fires;
 *   bit 3 (8)  tt_local_search_ordered got a dispatch order that is not a
 *              permutation of 0..P-1 (an entry out of range, or an entry seen
 *              twice: checked exactly on the device with a visited bitmap);
 *              out-of-range entries are skipped, a duplicated individual is
 *              searched twice concurrently (undefined result);
 *   bit 4 (16) the local search's per-stream redo list overflowed (unreachable:
 *              it holds P entries and a launch lists each wave at most once);
 *              the individuals not listed are left unsearched.
 * Synchronises the device. */
int tt_device_status(const tt_problem* p, int32_t* status);

const char* tt_last_error(void);
int tt_version(void);

#ifdef __cplusplus
}
#endif

#endif /* TTGA_H */

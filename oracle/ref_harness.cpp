// ref_harness — TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" shim over the reference's OWN Problem / Solution / Random
// objects (nelilepo/timetabling-ga-mpi-openmp, compiled unmodified from
// /root/reference by oracle/Makefile into oracle/_ref/libttref.so). Used to
// (1) generate the golden vectors committed under tests/golden/ and
// (2) time the reference's evaluation functions as bench.py's CPU baseline.
//
// Reference F1 (uninitialised busy[] VLA, Solution.cpp:778) is neutralised
// WITHOUT editing the sources: the Makefile compiles them with clang's
// -ftrivial-auto-var-init=zero, which zero-fills that VLA.
//
// Written in C++98 (the reference's Random.h needs gnu++98).
#include <algorithm>
#include <sstream>
#include <vector>
#include <sys/time.h>
#include <omp.h>

#include "Problem.h"
#include "Solution.h"
#include "Random.h"

typedef unsigned char u8;

static void load_solution(Solution* s, const u8* slot, const u8* room, int E) {
    // deserializeSolution-style construction (ga.cpp:344-368): sln pairs, then
    // timeslot_events built by ascending event index.
    for (int e = 0; e < E; e++) {
        s->sln[e].first = slot[e];
        s->sln[e].second = room ? room[e] : -1;
    }
    for (int e = 0; e < E; e++) s->timeslot_events[slot[e]].push_back(e);
}

static void store_solution(const Solution* s, u8* slot, u8* room, int E) {
    for (int e = 0; e < E; e++) {
        if (slot) slot[e] = (u8)s->sln[e].first;
        if (room) room[e] = (u8)s->sln[e].second;
    }
}

extern "C" {

// Builds a .tim text image and parses it with the reference's Problem(istream&).
void* ref_problem_create(int E, int R, int F, int S, const int* room_size, const int* A,
                         const int* room_feat, const int* event_feat) {
    std::ostringstream os;
    os << E << " " << R << " " << F << " " << S << "\n";
    for (int r = 0; r < R; r++) os << room_size[r] << "\n";
    for (long i = 0; i < (long)S * E; i++) os << A[i] << "\n";
    for (long i = 0; i < (long)R * F; i++) os << room_feat[i] << "\n";
    for (long i = 0; i < (long)E * F; i++) os << event_feat[i] << "\n";
    std::istringstream is(os.str());
    return new Problem(is);
}

void* ref_problem_from_tim(const char* path) {
    std::ifstream is(path);
    return new Problem(is);
}

void ref_problem_destroy(void* p) { delete (Problem*)p; }

void ref_problem_dims(const void* p, int* dims) {
    const Problem* P = (const Problem*)p;
    dims[0] = P->n_of_events; dims[1] = P->n_of_rooms; dims[2] = P->n_of_features; dims[3] = P->n_of_students;
}

void ref_problem_derived(const void* p, int* student_number, int* corr, int* possible) {
    const Problem* P = (const Problem*)p;
    const int E = P->n_of_events, R = P->n_of_rooms;
    for (int i = 0; i < E; i++) student_number[i] = P->studentNumber[i];
    for (int i = 0; i < E; i++)
        for (int j = 0; j < E; j++) corr[(long)i * E + j] = P->eventCorrelations[i][j];
    for (int i = 0; i < E; i++)
        for (int j = 0; j < R; j++) possible[(long)i * R + j] = P->possibleRooms[i][j];
}

void ref_problem_matrices(const void* p, int* room_size, int* A, int* room_feat, int* event_feat) {
    const Problem* P = (const Problem*)p;
    const int E = P->n_of_events, R = P->n_of_rooms, F = P->n_of_features, S = P->n_of_students;
    for (int r = 0; r < R; r++) room_size[r] = P->roomSize[r];
    for (int s = 0; s < S; s++)
        for (int e = 0; e < E; e++) A[(long)s * E + e] = P->student_events[s][e];
    for (int r = 0; r < R; r++)
        for (int f = 0; f < F; f++) room_feat[(long)r * F + f] = P->room_features[r][f];
    for (int e = 0; e < E; e++)
        for (int f = 0; f < F; f++) event_feat[(long)e * F + f] = P->event_features[e][f];
}

void ref_rand(long seed, int n, double* out, long* final_state) {
    Random r(0);
    r.seed = seed;
    for (int i = 0; i < n; i++) out[i] = r.next();
    *final_state = r.seed;
}

// computeFeasibility / computeHcv / computeScv / computePenalty per individual.
void ref_eval(void* p, const u8* slot, const u8* room, int np, int* hcv, int* scv, u8* feasible,
              int* penalty) {
    Problem* P = (Problem*)p;
    const int E = P->n_of_events;
    Random r(1);
    for (int i = 0; i < np; i++) {
        Solution s(P, &r);
        load_solution(&s, slot + (long)i * E, room + (long)i * E, E);
        feasible[i] = s.computeFeasibility() ? 1 : 0;
        hcv[i] = s.computeHcv();
        scv[i] = s.computeScv();
        penalty[i] = s.computePenalty();
    }
}

// CPU baseline: the same evaluation, OpenMP over individuals. Solutions are
// built before the clock starts; the timed region is exactly
// computeFeasibility + computeHcv + computeScv + penalty.
// Returns seconds.
double ref_eval_timed(void* p, const u8* slot, const u8* room, int np, int threads, int* hcv, int* scv,
                      u8* feasible, int* penalty) {
    Problem* P = (Problem*)p;
    const int E = P->n_of_events;
    Random r(1);
    std::vector<Solution*> pop(np);
    for (int i = 0; i < np; i++) {
        pop[i] = new Solution(P, &r);
        load_solution(pop[i], slot + (long)i * E, room + (long)i * E, E);
        for (int t = 0; t < 45; t++) pop[i]->timeslot_events[t];   // materialise all map keys
    }
    omp_set_num_threads(threads);
    struct timeval t0, t1;
    gettimeofday(&t0, 0);
#pragma omp parallel for schedule(dynamic, 4)
    for (int i = 0; i < np; i++) {
        Solution* s = pop[i];
        bool f = s->computeFeasibility();
        int h = s->computeHcv();
        int c = s->computeScv();
        hcv[i] = h;
        scv[i] = c;
        feasible[i] = f ? 1 : 0;
        penalty[i] = f ? c : 1000000 + h;
    }
    gettimeofday(&t1, 0);
    for (int i = 0; i < np; i++) delete pop[i];
    return (t1.tv_sec - t0.tv_sec) + 1e-6 * (t1.tv_usec - t0.tv_usec);
}

// assignRooms on every non-empty slot, ascending t.
void ref_assign_rooms(void* p, const u8* slot, u8* room, int np) {
    Problem* P = (Problem*)p;
    const int E = P->n_of_events;
    Random r(1);
    for (int i = 0; i < np; i++) {
        Solution s(P, &r);
        load_solution(&s, slot + (long)i * E, 0, E);
        for (int t = 0; t < 45; t++)
            if ((int)s.timeslot_events[t].size()) s.assignRooms(t);
        store_solution(&s, 0, room + (long)i * E, E);
    }
}

void ref_random_init(void* p, long* rng, u8* slot, u8* room, int np) {
    Problem* P = (Problem*)p;
    const int E = P->n_of_events;
    for (int i = 0; i < np; i++) {
        Random r(0);
        r.seed = rng[i];
        Solution s(P, &r);
        s.RandomInitialSolution();
        store_solution(&s, slot + (long)i * E, room + (long)i * E, E);
        rng[i] = r.seed;
    }
}

void ref_local_search(void* p, u8* slot, u8* room, long* rng, int np, int max_steps, double p1, double p2,
                      double p3) {
    Problem* P = (Problem*)p;
    const int E = P->n_of_events;
    for (int i = 0; i < np; i++) {
        Random r(0);
        r.seed = rng[i];
        Solution s(P, &r);
        load_solution(&s, slot + (long)i * E, room + (long)i * E, E);
        s.localSearch(max_steps, 999999, p1, p2, p3);
        store_solution(&s, slot + (long)i * E, room + (long)i * E, E);
        rng[i] = r.seed;
    }
}

// localSearch over a population, OpenMP over individuals (each with its own
// Random, so the result equals the serial ref_local_search). Returns seconds.
double ref_local_search_timed(void* p, u8* slot, u8* room, long* rng, int np, int max_steps, int threads) {
    Problem* P = (Problem*)p;
    const int E = P->n_of_events;
    omp_set_num_threads(threads);
    struct timeval t0, t1;
    gettimeofday(&t0, 0);
#pragma omp parallel for schedule(dynamic, 1)
    for (int i = 0; i < np; i++) {
        Random r(0);
        r.seed = rng[i];
        Solution s(P, &r);
        load_solution(&s, slot + (long)i * E, room + (long)i * E, E);
        s.localSearch(max_steps);
        store_solution(&s, slot + (long)i * E, room + (long)i * E, E);
        rng[i] = r.seed;
    }
    gettimeofday(&t1, 0);
    return (t1.tv_sec - t0.tv_sec) + 1e-6 * (t1.tv_usec - t0.tv_usec);
}

// Crossover into a FRESH child (no prior RandomInitialSolution), i.e. the
// reference's crossover without the F2 stale-list defect.
void ref_crossover(void* p, const u8* slot1, const u8* slot2, long* rng, u8* slot, u8* room, int np) {
    Problem* P = (Problem*)p;
    const int E = P->n_of_events;
    for (int i = 0; i < np; i++) {
        Random r(0);
        r.seed = rng[i];
        Solution a(P, &r), b(P, &r), c(P, &r);
        load_solution(&a, slot1 + (long)i * E, 0, E);
        load_solution(&b, slot2 + (long)i * E, 0, E);
        c.crossover(&a, &b);
        store_solution(&c, slot + (long)i * E, room + (long)i * E, E);
        rng[i] = r.seed;
    }
}

void ref_mutation(void* p, u8* slot, u8* room, long* rng, int np) {
    Problem* P = (Problem*)p;
    const int E = P->n_of_events;
    for (int i = 0; i < np; i++) {
        Random r(0);
        r.seed = rng[i];
        Solution s(P, &r);
        load_solution(&s, slot + (long)i * E, room + (long)i * E, E);
        s.mutation();
        store_solution(&s, slot + (long)i * E, room + (long)i * E, E);
        rng[i] = r.seed;
    }
}

// The per-child work of the reference's generation loop (ga.cpp:543-577),
// OpenMP over children, each child with its own Random: three
// RandomInitialSolution (child, copyParent1, copyParent2), two selection5
// tournaments over pop_penalty (restated from ga.cpp:129-145: first drawn wins
// ties), the parent copies, next() < 0.8 ? crossover : copy, next() < 0.5 ?
// mutation, localSearch(max_steps), computePenalty. as_is = 1: as in the
// reference, the crossover child is the one that already holds a random
// solution (F2: its timeslot lists then hold every event twice, which slows
// the matching and the local search); as_is = 0: crossover into a fresh
// Solution, the semantics the device engine implements.
// The parents are loaded with all 45 timeslot keys present, as every member
// of the reference's population has them (RandomInitialSolution touches each
// key, Solution.cpp:56-59), so copy() replaces every list of cp1/cp2.
// Outputs (any may be NULL): the child's slot/room rows, hcv, scv, feasible
// and penalty (computed after the clock stops) and its final RNG state.
// Returns the seconds of the per-child work.
double ref_ga_children(void* p, const u8* pop_slot, const u8* pop_room, const int* pop_penalty, int N, long* rng,
                       int C, int max_steps, int threads, int as_is, u8* out_slot, u8* out_room, int* out_hcv,
                       int* out_scv, u8* out_feasible, int* out_penalty) {
    Problem* P = (Problem*)p;
    const int E = P->n_of_events;
    const bool keep = out_slot || out_room || out_hcv || out_scv || out_feasible || out_penalty;
    std::vector<Solution*> kept(keep ? C : 0, (Solution*)0);
    std::vector<Solution*> owned(keep ? 3 * (long)C + C : 0, (Solution*)0);
    std::vector<Random*> rngs(C, (Random*)0);
    for (int c = 0; c < C; c++) {
        rngs[c] = new Random(0);
        rngs[c]->seed = rng[c];
    }
    omp_set_num_threads(threads);
    struct timeval t0, t1;
    gettimeofday(&t0, 0);
#pragma omp parallel for schedule(dynamic, 1)
    for (int c = 0; c < C; c++) {
        Random& r = *rngs[c];
        Solution* child = new Solution(P, &r);
        child->RandomInitialSolution();
        Solution* cp1 = new Solution(P, &r);
        cp1->RandomInitialSolution();
        Solution* cp2 = new Solution(P, &r);
        cp2->RandomInitialSolution();
        int sel[2];
        for (int k = 0; k < 2; k++) {
            int best = (int)(r.next() * N);
            for (int i = 1; i < 5; i++) {
                const int t = (int)(r.next() * N);
                if (pop_penalty[t] < pop_penalty[best]) best = t;
            }
            sel[k] = best;
        }
        Solution a(P, &r), b(P, &r);
        load_solution(&a, pop_slot + (long)sel[0] * E, pop_room + (long)sel[0] * E, E);
        load_solution(&b, pop_slot + (long)sel[1] * E, pop_room + (long)sel[1] * E, E);
        for (int t = 0; t < 45; t++) {
            a.timeslot_events[t];
            b.timeslot_events[t];
        }
        cp1->copy(&a);
        cp2->copy(&b);
        Solution* use = child;
        Solution* fresh = new Solution(P, &r);
        if (r.next() < 0.8) {
            if (as_is) child->crossover(cp1, cp2);
            else { fresh->crossover(cp1, cp2); use = fresh; }
        } else {
            use = cp1;
        }
        if (r.next() < 0.5) use->mutation();
        use->localSearch(max_steps);
        use->computePenalty();
        if (keep) {
            kept[c] = use;
            owned[4L * c] = child; owned[4L * c + 1] = cp1; owned[4L * c + 2] = cp2; owned[4L * c + 3] = fresh;
        } else {
            delete child;
            delete cp1;
            delete cp2;
            delete fresh;
        }
    }
    gettimeofday(&t1, 0);
    for (int c = 0; c < C; c++) {
        rng[c] = rngs[c]->seed;
        if (keep) {
            Solution* s = kept[c];
            store_solution(s, out_slot ? out_slot + (long)c * E : 0, out_room ? out_room + (long)c * E : 0, E);
            const bool f = s->computeFeasibility();
            const int h = s->computeHcv(), v = s->computeScv();
            if (out_hcv) out_hcv[c] = h;
            if (out_scv) out_scv[c] = v;
            if (out_feasible) out_feasible[c] = f ? 1 : 0;
            if (out_penalty) out_penalty[c] = s->penalty;
        }
        delete rngs[c];
    }
    for (size_t k = 0; k < owned.size(); k++) delete owned[k];
    return (t1.tv_sec - t0.tv_sec) + 1e-6 * (t1.tv_usec - t0.tv_usec);
}

// ref_ga_children without outputs: the bench's CPU baseline (seconds).
double ref_ga_children_timed(void* p, const u8* pop_slot, const u8* pop_room, const int* pop_penalty, int N,
                             long* rng, int C, int max_steps, int threads, int as_is) {
    return ref_ga_children(p, pop_slot, pop_room, pop_penalty, N, rng, C, max_steps, threads, as_is, 0, 0, 0, 0, 0,
                           0);
}

static bool by_penalty(Solution* a, Solution* b) { return a->penalty < b->penalty; }   // ga.cpp:150-153

// The value setCurrentCost logs for pop[0] (ga.cpp:203-228): scv if feasible,
// else computeHcv()*1e6 + computeScv() (which also refreshes both fields).
static long log_value(Solution* s) {
    if (s->feasible) return s->scv;
    const long h = s->computeHcv();
    return h * 1000000L + s->computeScv();
}

// Whole single-island GA runs of the reference, one per seed, for the
// statistical comparison of GA trajectories (tools/ga_quality.py). Each run is
// ga.cpp with one MPI rank and one OpenMP thread (-c 1), restated around the
// reference's own Solution objects: Random(seed) (ga.cpp:400-401); pop_size
// members RandomInitialSolution + localSearch(max_steps) + computePenalty
// (:429-434); then generations 0..gens-1 (ga.cpp runs gens = 2001,
// :504), each: three RandomInitialSolution, two selection5 (:129-145),
// next() < 0.8 ? crossover : copy of parent 1, next() < 0.5 ? mutation,
// localSearch, computePenalty, pop[N-1]->copy(child), std::sort (:543-585).
// as_is = 1 keeps F2 (crossover into the child that already holds a random
// solution, as ga.cpp:543-563); as_is = 0 crosses into a fresh Solution.
// No migration (one island). Runs are independent: OpenMP over seeds.
// Outputs per run: best hcv, scv, feasible, penalty after the last
// generation (hcv recomputed, as endTry does, ga.cpp:189), and trace[run][g] =
// the value setCurrentCost logs for pop[0] after generation g (g = 0: the
// sorted initial population).
double ref_ga_run(void* p, const long* seeds, int runs, int pop_size, int gens, int max_steps, int as_is,
                  int threads, int* hcv, int* scv, u8* feasible, int* penalty, long* trace) {
    Problem* P = (Problem*)p;
    omp_set_num_threads(threads);
    struct timeval t0, t1;
    gettimeofday(&t0, 0);
#pragma omp parallel for schedule(dynamic, 1)
    for (int k = 0; k < runs; k++) {
        Random rnd(seeds[k]);
        std::vector<Solution*> pop(pop_size);
        for (int i = 0; i < pop_size; i++) {
            pop[i] = new Solution(P, &rnd);
            pop[i]->RandomInitialSolution();
            pop[i]->localSearch(max_steps);
            pop[i]->computePenalty();
        }
        std::sort(pop.begin(), pop.end(), by_penalty);
        long* tr = trace ? trace + (long)k * (gens + 1) : 0;
        const long v0 = log_value(pop[0]);
        if (tr) tr[0] = v0;
        for (int g = 0; g < gens; g++) {
            Solution* child = new Solution(P, &rnd);
            child->RandomInitialSolution();
            Solution* cp1 = new Solution(P, &rnd);
            cp1->RandomInitialSolution();
            Solution* cp2 = new Solution(P, &rnd);
            cp2->RandomInitialSolution();
            Solution* sel[2];
            for (int s = 0; s < 2; s++) {
                int best = (int)(rnd.next() * pop_size);
                for (int i = 1; i < 5; i++) {
                    const int t = (int)(rnd.next() * pop_size);
                    if (pop[t]->penalty < pop[best]->penalty) best = t;
                }
                sel[s] = pop[best];
            }
            cp1->copy(sel[0]);
            cp2->copy(sel[1]);
            Solution* use = child;
            Solution* fresh = 0;
            if (rnd.next() < 0.8) {
                if (as_is) child->crossover(cp1, cp2);
                else { fresh = new Solution(P, &rnd); fresh->crossover(cp1, cp2); use = fresh; }
            } else {
                use = cp1;
            }
            if (rnd.next() < 0.5) use->mutation();
            use->localSearch(max_steps);
            use->computePenalty();
            pop[pop_size - 1]->copy(use);
            std::sort(pop.begin(), pop.end(), by_penalty);
            const long v = log_value(pop[0]);
            if (tr) tr[g + 1] = v;
            delete child;
            delete cp1;
            delete cp2;
            delete fresh;
        }
        hcv[k] = pop[0]->computeHcv();
        scv[k] = pop[0]->computeScv();
        feasible[k] = pop[0]->feasible ? 1 : 0;
        penalty[k] = pop[0]->penalty;
        for (int i = 0; i < pop_size; i++) delete pop[i];
    }
    gettimeofday(&t1, 0);
    return (t1.tv_sec - t0.tv_sec) + 1e-6 * (t1.tv_usec - t0.tv_usec);
}

}  // extern "C"

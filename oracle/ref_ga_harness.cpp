// ref_ga_harness — TEST INFRASTRUCTURE ONLY.
//
// Drives the reference's OWN ga.cpp functions (compiled unmodified from
// /root/reference by oracle/Makefile into oracle/_ref/libttref_ga.so, with
// -Dmain=ref_ga_main so its main is not the program's) and its vendored
// jsoncpp, to pin two things to reference code instead of restatements:
//
//  * the JSON lines of setCurrentCost (ga.cpp:203-228), setGlobalCost
//    (:234-257), endTry (:169-197) and the final runEntry (:603-609), written
//    by jsoncpp's own writeString (jsoncpp.cpp:5080) -> tests/golden/json_lines.json;
//  * selection5 (ga.cpp:129-145) and compareSolution/std::sort (:150-153,583)
//    on populations of the reference's own Solution objects.
//
// ga.cpp needs MPI (setGlobalCost's MPI_Allreduce): the harness initialises
// MPICH as a singleton (one process, no mpiexec).
#include <algorithm>
#include <sstream>
#include <string>
#include <vector>

#include <mpi.h>

#include "Problem.h"
#include "Solution.h"
#include "Random.h"
#include "json/json.h"

using namespace Json;

// ga.cpp globals and functions (external linkage in ga.cpp)
extern ostream* os;
extern Random* rnd;
extern int id;
extern int p;
extern int tid;
Solution* selection5(Solution** pop, int popSize);
bool compareSolution(Solution* sol1, Solution* sol2);
void beginTry();
void endTry(Solution* bestSolution, Value solution);
void setCurrentCost(Solution* currentSolution, int tid, StreamWriterBuilder swb, Value logEntry);
void setGlobalCost(Solution* currentSolution, StreamWriterBuilder swb, Value runEntry);

typedef unsigned char u8;

static void ensure_mpi() {
    int ok = 0;
    MPI_Initialized(&ok);
    if (!ok) {
        int argc = 0;
        char** argv = 0;
        MPI_Init(&argc, &argv);
        MPI_Comm_size(MPI_COMM_WORLD, &p);
        MPI_Comm_rank(MPI_COMM_WORLD, &id);
    }
}

// deserializeSolution-style construction (ga.cpp:344-368) + the fields the
// reference computes for a population member (computePenalty, ga.cpp:433,577)
static Solution* make_solution(Problem* P, Random* r, const u8* slot, const u8* room) {
    Solution* s = new Solution(P, r);
    const int E = P->n_of_events;
    for (int e = 0; e < E; e++) {
        s->sln[e].first = slot[e];
        s->sln[e].second = room[e];
    }
    for (int e = 0; e < E; e++) s->timeslot_events[slot[e]].push_back(e);
    s->computePenalty();
    s->hcv = s->computeHcv();
    s->scv = s->computeScv();
    return s;
}

static int copy_out(const std::string& s, char* out, int cap) {
    const int n = (int)s.size();
    if (out && cap > 0) {
        const int m = n < cap - 1 ? n : cap - 1;
        std::copy(s.begin(), s.begin() + m, out);
        out[m] = 0;
    }
    return n;
}

extern "C" {

// jsoncpp's rendering of one double (the "time"/"totalTime" fields): the
// object {"x": v} through writeString with indentation "" (ga.cpp:170-171).
int refga_json_double(double v, char* out, int cap) {
    StreamWriterBuilder swb;
    swb.settings_["indentation"] = "";
    Value x;
    x["x"] = v;
    return copy_out(writeString(swb, x), out, cap);
}

// The JSON lines one island of the reference writes when its pop[0] takes the
// values of individuals 0..n-1 in turn: beginTry (ga.cpp:163-167), then per
// step setCurrentCost(pop[0], tids[i]) (the logEntry of :203-228, procID =
// proc), then setGlobalCost(pop[0]) (:234-257, one MPI rank), endTry(pop[0])
// (:169-197) and the final runEntry of main (:603-609, procsNum = 1,
// threadsNum = threads). Lines are '\n'-separated; returns the length.
int refga_log_lines(void* problem, const u8* slot, const u8* room, int n, const int* tids, int proc, int threads,
                    char* out, int cap) {
    ensure_mpi();
    Problem* P = (Problem*)problem;
    const int E = P->n_of_events;
    Random r(1);
    std::ostringstream buf;
    ostream* saved = os;
    os = &buf;
    id = proc;
    tid = 0;
    StreamWriterBuilder swb;
    swb.settings_["indentation"] = "";
    beginTry();
    Value logEntry;
    logEntry["logEntry"]["procID"] = proc;                 // ga.cpp:502
    std::vector<Solution*> seen;
    for (int i = 0; i < n; i++) {
        Solution* s = make_solution(P, &r, slot + (size_t)i * E, room + (size_t)i * E);
        seen.push_back(s);
        setCurrentCost(s, tids[i], swb, logEntry);
    }
    Solution* last = seen.back();
    Value runEntry, solution;
    solution["solution"]["procID"] = proc;                 // ga.cpp:474
    setGlobalCost(last, swb, runEntry);
    endTry(last, solution);
    runEntry["runEntry"]["procsNum"] = 1;                  // ga.cpp:603-608 (main's own runEntry is
    runEntry["runEntry"]["threadsNum"] = threads;          // untouched by setGlobalCost: by value)
    runEntry["runEntry"]["totalTime"] = 0.5;
    buf << writeString(swb, runEntry) << std::endl;
    os = saved;
    for (size_t k = 0; k < seen.size(); k++) delete seen[k];
    return copy_out(buf.str(), out, cap);
}

// selection5 (ga.cpp:129-145) over a population of the reference's own
// Solution objects with the given penalties, drawing from Random(seed):
// writes `draws` winners (indices) and the final RNG state.
void refga_selection5(void* problem, const int* penalty, int N, long seed, int draws, int* winners, long* state) {
    Problem* P = (Problem*)problem;
    Random r(1);
    r.seed = seed;
    std::vector<Solution*> pop(N);
    for (int i = 0; i < N; i++) {
        pop[i] = new Solution(P, &r);
        pop[i]->penalty = penalty[i];
    }
    Random* saved = rnd;
    rnd = &r;
    for (int k = 0; k < draws; k++) {
        Solution* w = selection5(&pop[0], N);
        winners[k] = (int)(std::find(pop.begin(), pop.end(), w) - pop.begin());
    }
    rnd = saved;
    *state = r.seed;
    for (int i = 0; i < N; i++) delete pop[i];
}

// std::sort(pop, pop + N, compareSolution) (ga.cpp:583): the penalties in
// sorted order (positions of equal penalties are unspecified there).
void refga_sort_penalties(void* problem, int* penalty, int N) {
    Problem* P = (Problem*)problem;
    Random r(1);
    std::vector<Solution*> pop(N);
    for (int i = 0; i < N; i++) {
        pop[i] = new Solution(P, &r);
        pop[i]->penalty = penalty[i];
    }
    std::sort(pop.begin(), pop.end(), compareSolution);
    for (int i = 0; i < N; i++) {
        penalty[i] = pop[i]->penalty;
        delete pop[i];
    }
}

}  // extern "C"

// ttga-ga: the reference's ga.cpp driver (ga.cpp:370-613) as a native host
// program over the C-ABI of include/ttga.h. One island per GPU of this node;
// the MPI island model becomes RCCL over xGMI (one host thread and one
// communicator rank per GPU, ncclCommInitAll), the OpenMP threads of a rank
// become C children bred per batched generation. With --islands K != --gpus,
// island g runs on GPU g % gpus and migrants move by device copies (the same
// ring, no communicator): K islands can share one GPU. --rccl takes the RCCL
// path for one island on one GPU too (a one-rank communicator: the ring's
// send/recv pairs go to the rank itself), so the communicator's calls run on a
// one-GPU box.
//
//   ttga-ga -i instance.tim [-s seed] [-p type] [-c children]
//           [-p1 x -p2 y -p3 z] [--gpus G] [--islands K] [--pop N] [--generations n] [--rccl] [--stagger]
//
// --stagger / --stagger-parts P: the children of a generation are 2 / P
// sub-batches on as many streams, sub-batch h bred from the population after
// the replacement of sub-batch h - P (ttga/ga.py Island, schedule "staggered";
// same results as the Python driver with the same option).
//
// Reference correspondence:
//  * CLI: `-key value` pairs and messages of Control::Control (Control.cpp:3-137);
//    -o -n -t -m -l are parsed and echoed, then ignored, as in ga.cpp (output
//    always goes to stdout, ga.cpp:60).
//  * -p -> maxSteps 200 / 1000 / 2000 (ga.cpp:389-397).
//  * island k runs with seed abs(seed + k*(seed/10)) (ga.cpp:412); all islands
//    start from island 0's initial population (ga.cpp:429-444,463-464).
//  * generation loop, migration before generations g with (g+1) % 100 == 50,
//    best -> right neighbour's pop[N-1], 2nd best -> left neighbour's pop[N-2]
//    (ga.cpp:479-540); MIN all-reduce of the best value (ga.cpp:234-257);
//    JSON lines of endTry / setCurrentCost / runEntry (ga.cpp:169-228,602-609)
//    in jsoncpp's compact format (sorted keys, doubles as %.17g); logEntry
//    threadID = the child slot whose replacement made the new best (ga.cpp:584);
//    logEntry/solution times from beginTry (ga.cpp:476), the last totalTime
//    from process start (ga.cpp:381).
//  * same stream layout as ttga/ga.py (Island): member i of the initial
//    population draws from Random(|s|+1+i), child slot c from Random(|s|+1+N+c).
#include <rccl/rccl.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <iostream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ttga.h"

namespace {

[[noreturn]] void die(const std::string& msg) {
    std::cerr << "ttga-ga: " << msg << std::endl;
    std::exit(1);
}

void check_tt(int rc, const char* what) {
    if (rc != TT_OK) die(std::string(what) + ": " + tt_last_error());
}

void check_hip(hipError_t e, const char* what) {
    if (e != hipSuccess) die(std::string(what) + ": " + hipGetErrorString(e));
}

void check_nccl(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) die(std::string(what) + ": " + ncclGetErrorString(r));
}

// ---------------------------------------------------------------- Control
const char* kUsage = " -i InputFile [-o OutputFile] [-n NumberOfTries] [-s RandomSeed] [-t TimeLimit] [-p ProblemType]";

struct Control {
    int threads = 1, tries = 10, problem_type = 1, max_steps = 100;
    double time_limit = 90, ls_limit = 99999, p1 = 1.0, p2 = 1.0, p3 = 0.0;
    long seed = 0;
    std::string input, output;
    int gpus = 1, islands = 0, pop = 10, generations = -1;
    bool rccl = false;
    int stagger = 0;                              // sub-batches of the staggered schedule (0: batch)
};

// Control::Control (Control.cpp:3-137) plus the --gpus/--pop/--generations extensions.
Control parse_control(int argc, char** argv) {
    std::vector<std::string> args(argv + 1, argv + argc);
    Control c;
    if (auto it = std::find(args.begin(), args.end(), "--rccl"); it != args.end()) {
        c.rccl = true;
        args.erase(it);
    }
    if (auto it = std::find(args.begin(), args.end(), "--stagger"); it != args.end()) {
        c.stagger = 2;
        args.erase(it);
    }
    for (const char* k : {"--gpus", "--islands", "--pop", "--generations", "--children", "--stagger-parts"}) {
        auto it = std::find(args.begin(), args.end(), k);
        if (it != args.end()) {
            if (it + 1 == args.end()) die(std::string("missing value for ") + k);
            const int v = std::atoi((it + 1)->c_str());
            if (!std::strcmp(k, "--gpus")) c.gpus = v;
            else if (!std::strcmp(k, "--islands")) c.islands = v;
            else if (!std::strcmp(k, "--pop")) c.pop = v;
            else if (!std::strcmp(k, "--generations")) c.generations = v;
            else if (!std::strcmp(k, "--stagger-parts")) c.stagger = v;
            else c.threads = v;
            args.erase(it, it + 2);
        }
    }
    if (args.empty() || args.size() % 2 != 0) {
        std::cerr << "Parse error: Number of command line parameters incorrect\n";
        std::cerr << "Usage:" << std::endl << argv[0] << kUsage << std::endl;
        std::exit(1);
    }
    std::map<std::string, std::string> kv;
    for (size_t i = 0; i + 1 < args.size(); i += 2) kv[args[i]] = args[i + 1];
    auto has = [&](const char* k) { return kv.count(k) > 0; };
    if (has("-c")) {
        c.threads = std::atoi(kv["-c"].c_str());
        std::cout << "Max number of threads " << c.threads << std::endl;
    } else {
        std::cerr << "Warning: Number of threads is set to default (1)" << std::endl;
    }
    if (!has("-i")) {
        std::cerr << "Error: No input file given, exiting" << std::endl;
        std::cerr << "Usage:" << std::endl << argv[0] << kUsage << std::endl;
        std::exit(1);
    }
    c.input = kv["-i"];
    if (has("-o")) c.output = kv["-o"];
    else std::cerr << "Warning: No output file given, writing to stdout" << std::endl;
    if (has("-n")) {
        c.tries = std::atoi(kv["-n"].c_str());
        std::cout << "Max number of tries " << c.tries << std::endl;
    } else {
        std::cerr << "Warning: Number of tries is set to default (10)" << std::endl;
    }
    if (has("-t")) {
        c.time_limit = std::atof(kv["-t"].c_str());
        std::cout << "Time limit " << c.time_limit << std::endl;
    } else {
        std::cerr << "Warning: Time limit is set to default (90 sec)" << std::endl;
    }
    if (has("-p")) {
        c.problem_type = std::atoi(kv["-p"].c_str());
        std::cout << "Problem instance type " << c.problem_type << std::endl;
    }
    if (has("-m")) {
        c.max_steps = std::atoi(kv["-m"].c_str());
        std::cout << "Max number of steps in the local search " << c.max_steps << std::endl;
    }
    if (has("-l")) {
        c.ls_limit = std::atof(kv["-l"].c_str());
        std::cout << "Local search time limit " << c.ls_limit << std::endl;
    } else {
        std::cerr << "Warning: The local search time limit is set to default (99999 sec)" << std::endl;
    }
    struct P { const char* key; double* dst; const char* dflt; int n; };
    for (P p : {P{"-p1", &c.p1, "1.0", 1}, P{"-p2", &c.p2, "1.0", 2}, P{"-p3", &c.p3, "0.0", 3}}) {
        if (has(p.key)) {
            *p.dst = std::atof(kv[p.key].c_str());
            std::cout << "LS move " << p.n << " probability " << *p.dst << std::endl;
        } else {
            std::cerr << "Warning: The local search move " << p.n << " probability is set to default " << p.dflt
                      << std::endl;
        }
    }
    if (has("-s")) {
        c.seed = std::atol(kv["-s"].c_str());
    } else {
        c.seed = (long)std::time(nullptr);
        std::cerr << "Warning: " << c.seed << " used as default random seed" << std::endl;
    }
    return c;
}

// ga.cpp:389-397
int max_steps_for(int problem_type) { return problem_type == 1 ? 200 : problem_type == 2 ? 1000 : 2000; }

// ga.cpp:412 (C int division)
long island_seed(long seed, int k) { return std::labs(seed + k * (seed / 10)); }

// ---------------------------------------------------------------- .tim
struct Instance {
    int E = 0, R = 0, F = 0, S = 0;
    std::vector<int32_t> room_size, student_events, room_features, event_features;
};

// Problem::Problem(istream&) token order (Problem.cpp:7-74).
Instance read_tim(const std::string& path) {
    std::ifstream in(path);
    if (!in) die("cannot open " + path);
    Instance t;
    if (!(in >> t.E >> t.R >> t.F >> t.S)) die("truncated .tim header in " + path);
    auto read = [&](std::vector<int32_t>& v, long n) {
        v.resize(n);
        for (long i = 0; i < n; i++)
            if (!(in >> v[i])) die("truncated .tim body in " + path);
    };
    read(t.room_size, t.R);
    read(t.student_events, (long)t.S * t.E);
    read(t.room_features, (long)t.R * t.F);
    read(t.event_features, (long)t.E * t.F);
    return t;
}

// ---------------------------------------------------------------- JSON
// jsoncpp StreamWriterBuilder with indentation "" (ga.cpp:170-171): compact,
// keys in std::map order, doubles "%.17g" (jsoncpp.cpp:4036-4068).
struct Json {
    enum Kind { Int, Bool, Real, Arr, Obj } kind = Obj;
    long i = 0;
    double d = 0;
    std::vector<long> arr;
    std::map<std::string, Json> obj;
    static Json I(long v) { Json j; j.kind = Int; j.i = v; return j; }
    static Json B(bool v) { Json j; j.kind = Bool; j.i = v; return j; }
    static Json D(double v) { Json j; j.kind = Real; j.d = v; return j; }
    static Json A(std::vector<long> v) { Json j; j.kind = Arr; j.arr = std::move(v); return j; }
    std::string str() const {
        char buf[40];
        switch (kind) {
            case Int: return std::to_string(i);
            case Bool: return i ? "true" : "false";
            case Real:
                if (std::isnan(d)) return "null";
                if (std::isinf(d)) return d < 0 ? "-1e+9999" : "1e+9999";
                std::snprintf(buf, sizeof buf, "%.17g", d);
                return buf;
            case Arr: {
                std::string s = "[";
                for (size_t k = 0; k < arr.size(); k++) s += (k ? "," : "") + std::to_string(arr[k]);
                return s + "]";
            }
            case Obj: {
                std::string s = "{";
                bool first = true;
                for (auto& kvp : obj) {
                    s += (first ? "\"" : ",\"") + kvp.first + "\":" + kvp.second.str();
                    first = false;
                }
                return s + "}";
            }
        }
        return "";
    }
};

Json wrap(const char* key, Json inner) {
    Json j;
    j.obj[key] = std::move(inner);
    return j;
}

// The four JSON line kinds of ga.cpp, shared by the driver and --replay-log.
// setCurrentCost state (ga.cpp:57-58, reset by beginTry :163-167) and decision (:203-228):
// feasible pop[0] logs when its scv differs from the last logged best,
// infeasible when hcv*1e6+scv is lower.
struct CostState {
    long best_scv = INT_MAX, best_eval = INT_MAX;
    bool offer(bool feasible, int scv, int hcv, long& entry) {
        if (feasible) {
            if (scv == best_scv) return false;
            best_scv = best_eval = entry = scv;
            return true;
        }
        const long ev = (long)hcv * 1000000 + scv;
        if (ev >= best_eval) return false;
        best_eval = entry = ev;
        return true;
    }
};

Json log_line(long best, int proc, int thread, double t) {
    Json e;
    e.obj["best"] = Json::I(best);
    e.obj["procID"] = Json::I(proc);
    e.obj["threadID"] = Json::I(thread);
    e.obj["time"] = Json::D(std::max(0.0, t));
    return wrap("logEntry", e);
}

// setGlobalCost (ga.cpp:234-257), printed by rank 0
Json run_best_line(bool feasible, long total_best) {
    Json r;
    r.obj["feasible"] = Json::B(feasible);
    r.obj["totalBest"] = Json::I(total_best);
    return wrap("runEntry", r);
}

// endTry (ga.cpp:169-197); threadID is the global tid, 0 outside the parallel region
Json solution_line(bool feasible, int scv, int hcv, const std::vector<uint8_t>& sl, const std::vector<uint8_t>& rm,
                   int proc, double t) {
    Json s;
    s.obj["feasible"] = Json::B(feasible);
    s.obj["procID"] = Json::I(proc);
    s.obj["threadID"] = Json::I(0);
    s.obj["totalTime"] = Json::D(t);
    if (feasible) {
        s.obj["totalBest"] = Json::I(scv);
        s.obj["timeslots"] = Json::A(std::vector<long>(sl.begin(), sl.end()));
        s.obj["rooms"] = Json::A(std::vector<long>(rm.begin(), rm.end()));
    } else {
        s.obj["totalBest"] = Json::I((long)hcv * 1000000 + scv);
    }
    return wrap("solution", s);
}

// main's closing runEntry (ga.cpp:603-609)
Json run_final_line(int procs, int threads, double t) {
    Json r;
    r.obj["procsNum"] = Json::I(procs);
    r.obj["threadsNum"] = Json::I(threads);
    r.obj["totalTime"] = Json::D(t);
    return wrap("runEntry", r);
}

// ttga-ga --replay-log FILE: the lines one island prints when its pop[0] takes
// the given values in turn (no GPU involved; tests/test_json_parity.py checks
// them against the reference's own ga.cpp + jsoncpp). FILE: "proc threads n E",
// n lines "feasible scv hcv tid", then the last member's E slots and E rooms.
// Times print as 0 (the last runEntry: 0.5).
int replay_log(const char* path) {
    std::ifstream in(path);
    if (!in) die(std::string("cannot open ") + path);
    int proc = 0, threads = 1, n = 0, E = 0;
    if (!(in >> proc >> threads >> n >> E) || n < 1 || E < 0) die("bad replay header");
    CostState cs;
    int f = 0, scv = 0, hcv = 0, tid = 0;
    for (int i = 0; i < n; i++) {
        if (!(in >> f >> scv >> hcv >> tid)) die("truncated replay file");
        long entry = 0;
        if (cs.offer(f != 0, scv, hcv, entry)) std::cout << log_line(entry, proc, tid, 0.0).str() << "\n";
    }
    std::vector<uint8_t> sl(E), rm(E);
    for (int e = 0; e < E; e++) { int v; in >> v; sl[e] = (uint8_t)v; }
    for (int e = 0; e < E; e++) { int v; in >> v; rm[e] = (uint8_t)v; }
    if (!in) die("truncated replay file");
    if (proc == 0) std::cout << run_best_line(f != 0, f ? scv : (long)hcv * 1000000 + scv).str() << "\n";
    std::cout << solution_line(f != 0, scv, hcv, sl, rm, proc, 0.0).str() << "\n";
    std::cout << run_final_line(1, threads, 0.5).str() << std::endl;
    return 0;
}

// ---------------------------------------------------------------- islands
struct Pop {
    int n = 0, E = 0;
    uint8_t *slot = nullptr, *room = nullptr, *feasible = nullptr;
    int32_t *hcv = nullptr, *scv = nullptr, *penalty = nullptr;
    void alloc(int n_, int E_) {
        n = n_; E = E_;
        check_hip(hipMalloc(&slot, (size_t)n * E), "hipMalloc");
        check_hip(hipMalloc(&room, (size_t)n * E), "hipMalloc");
        check_hip(hipMalloc(&feasible, (size_t)n), "hipMalloc");
        check_hip(hipMalloc(&hcv, 4 * (size_t)n), "hipMalloc");
        check_hip(hipMalloc(&scv, 4 * (size_t)n), "hipMalloc");
        check_hip(hipMalloc(&penalty, 4 * (size_t)n), "hipMalloc");
        check_hip(hipMemset(slot, 0, (size_t)n * E), "hipMemset");
        check_hip(hipMemset(room, 0, (size_t)n * E), "hipMemset");
    }
    void release() {
        for (void* p : {(void*)slot, (void*)room, (void*)feasible, (void*)hcv, (void*)scv, (void*)penalty})
            if (p) (void)hipFree(p);
    }
};

struct Member { bool feasible; int scv, hcv, penalty; };

class Output {
public:
    explicit Output(std::ostream& os) : os_(os) {}
    void line(const Json& j) {
        std::lock_guard<std::mutex> g(mu_);
        os_ << j.str() << std::endl;
    }
private:
    std::ostream& os_;
    std::mutex mu_;
};

double seconds_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

struct Island {
    int id = 0, device = 0, N = 0, C = 0, E = 0, max_steps = 0;
    long seed = 0;
    double p1 = 1, p2 = 1, p3 = 0, p_cross = 0.8, p_mut = 0.5;
    tt_problem* tp = nullptr;
    hipStream_t st = nullptr;
    Pop pop, child;
    int64_t *rng_init = nullptr, *rng_child = nullptr;
    uint8_t* flags = nullptr;
    void* work = nullptr;
    int32_t* order = nullptr;                         // LPT dispatch order (C >= kLptMinChildren)
    static constexpr int kLptMinChildren = 4096;      // as ttga.ga.Island
    // migrants (ga.cpp:318-335): slot[E] room[E] hcv scv penalty feasible
    uint8_t *send_best = nullptr, *send_second = nullptr, *recv_buf = nullptr;
    size_t migrant_bytes = 0;
    CostState cost;                                   // setCurrentCost state (ga.cpp:163-167)
    // staggered schedule (ttga.ga.Island schedule "staggered"): part j of the child
    // rows [off, off + n) on stream hs[j] with its own work buffer; every population
    // operation (breed or replace) waits for the previous one (ev_op), so sub-batch h
    // is bred after the replacement of h - parts and h - parts + 1 is replaced after
    // the breed of h
    int parts = 1;
    struct Part { int off = 0, n = 0; hipStream_t s = nullptr; void* work = nullptr; };
    std::vector<Part> part;
    hipEvent_t ev_op = nullptr;
    std::vector<int> pending;                         // parts searched, not yet replaced (breed order)
    int last_replace = 0;

    void setup(const Instance& inst) {
        check_hip(hipSetDevice(device), "hipSetDevice");
        check_tt(tt_problem_create(inst.E, inst.R, inst.F, inst.S, inst.room_size.data(), inst.student_events.data(),
                                   inst.room_features.data(), inst.event_features.data(), device, &tp),
                 "tt_problem_create");
        E = inst.E;
        check_hip(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
        pop.alloc(N, E);
        child.alloc(C, E);
        std::vector<int64_t> s(N + C);
        for (int k = 0; k < N + C; k++) s[k] = std::labs(seed) + 1 + k;     // ttga/ga.py stream_seeds
        check_hip(hipMalloc(&rng_init, 8 * (size_t)N), "hipMalloc");
        check_hip(hipMalloc(&rng_child, 8 * (size_t)C), "hipMalloc");
        check_hip(hipMemcpy(rng_init, s.data(), 8 * (size_t)N, hipMemcpyHostToDevice), "hipMemcpy");
        check_hip(hipMemcpy(rng_child, s.data() + N, 8 * (size_t)C, hipMemcpyHostToDevice), "hipMemcpy");
        check_hip(hipMalloc(&flags, (size_t)C), "hipMalloc");
        if (C >= kLptMinChildren) check_hip(hipMalloc(&order, 4 * (size_t)C), "hipMalloc");
        check_hip(hipMalloc(&work, std::max<size_t>(tt_ga_work_bytes(N, E), 16)), "hipMalloc");
        migrant_bytes = 2 * (size_t)E + 13;
        check_hip(hipMalloc(&send_best, migrant_bytes), "hipMalloc");
        check_hip(hipMalloc(&send_second, migrant_bytes), "hipMalloc");
        check_hip(hipMalloc(&recv_buf, 2 * migrant_bytes), "hipMalloc");
        if (parts > 1) {
            check_hip(hipEventCreateWithFlags(&ev_op, hipEventDisableTiming), "hipEventCreate");
            part.resize(parts);
            for (int j = 0, off = 0; j < parts; j++) {          // numpy.array_split's sizes
                const int n = C / parts + (j < C % parts ? 1 : 0);
                part[j].off = off;
                part[j].n = n;
                off += n;
                if (j == 0) {
                    part[j].s = st;
                    part[j].work = work;
                } else {
                    check_hip(hipStreamCreateWithFlags(&part[j].s, hipStreamNonBlocking), "hipStreamCreate");
                    check_hip(hipMalloc(&part[j].work, std::max<size_t>(tt_ga_work_bytes(N, E), 16)), "hipMalloc");
                }
            }
        }
    }

    void evaluate(Pop& p, hipStream_t s = nullptr) {
        check_tt(tt_eval(tp, p.slot, p.room, p.n, p.hcv, p.scv, p.feasible, p.penalty, s ? s : st), "tt_eval");
    }

    // ga.cpp:429-434 for every member, then the population is sorted
    void initialize() {
        check_tt(tt_random_init(tp, rng_init, pop.slot, pop.room, N, st), "tt_random_init");
        check_tt(tt_local_search_eval(tp, pop.slot, pop.room, rng_init, N, max_steps, p1, p2, p3, nullptr, pop.hcv,
                                      pop.scv, pop.feasible, pop.penalty, st),
                 "tt_local_search_eval");
        check_tt(tt_ga_replace(tp, pop.slot, pop.room, pop.hcv, pop.scv, pop.feasible, pop.penalty, N, pop.slot,
                               pop.room, pop.hcv, pop.scv, pop.feasible, pop.penalty, 0, work, st),
                 "tt_ga_replace");
        if (parts > 1) check_hip(hipEventRecord(ev_op, st), "hipEventRecord");
    }

    // children rows [off, off + n) as a population view
    Pop child_rows(int off, int n) const {
        Pop v;
        v.n = n; v.E = E;
        v.slot = child.slot + (size_t)off * E; v.room = child.room + (size_t)off * E;
        v.feasible = child.feasible + off; v.hcv = child.hcv + off; v.scv = child.scv + off;
        v.penalty = child.penalty + off;
        return v;
    }

    // breed n children into rows [off, off + n) on stream s
    void breed(int off, int n, hipStream_t s) {
        Pop c = child_rows(off, n);
        check_tt(tt_ga_breed(tp, pop.slot, pop.room, pop.penalty, N, rng_child + off, n, p_cross, p_mut, 1, c.slot,
                             c.room, flags + off, s),
                 "tt_ga_breed");
    }

    // LPT order (C >= kLptMinChildren), localSearch and evaluation of rows [off, off + n) on s
    // (the search and the evaluation in one launch: ga.cpp:574-575)
    void search(int off, int n, hipStream_t s, void* w) {
        Pop c = child_rows(off, n);
        const int32_t* ord = nullptr;
        if (order) {
            // longest-expected first: the children's hcv before the search, descending
            // (a generation's search launch ends with its slowest children); same results
            evaluate(c, s);
            check_tt(tt_lpt_order(tp, c.hcv, n, order + off, w, s), "tt_lpt_order");
            ord = order + off;
        }
        check_tt(tt_local_search_eval(tp, c.slot, c.room, rng_child + off, n, max_steps, p1, p2, p3, ord, c.hcv, c.scv,
                                      c.feasible, c.penalty, s),
                 "tt_local_search_eval");
    }

    void replace(int off, int n, hipStream_t s, void* w) {
        Pop c = child_rows(off, n);
        check_tt(tt_ga_replace(tp, pop.slot, pop.room, pop.hcv, pop.scv, pop.feasible, pop.penalty, N, c.slot, c.room,
                               c.hcv, c.scv, c.feasible, c.penalty, n, w, s),
                 "tt_ga_replace");
    }

    // one generation of C children (ga.cpp:543-585)
    void step() {
        if (parts > 1) {
            for (int j = 0; j < parts; j++) part_step(j);
            return;
        }
        breed(0, C, st);
        search(0, C, st, work);
        replace(0, C, st, work);
    }

    void part_step(int j) {
        const Part& p = part[j];
        check_hip(hipStreamWaitEvent(p.s, ev_op, 0), "hipStreamWaitEvent");      // breed(h) after replace(h - parts)
        breed(p.off, p.n, p.s);
        check_hip(hipEventRecord(ev_op, p.s), "hipEventRecord");
        if ((int)pending.size() >= parts - 1) replace_oldest();                 // replace(h - parts + 1) after breed(h)
        search(p.off, p.n, p.s, p.work);
        pending.push_back(j);
    }

    void replace_oldest() {
        const int j = pending.front();
        pending.erase(pending.begin());
        const Part& p = part[j];
        check_hip(hipStreamWaitEvent(p.s, ev_op, 0), "hipStreamWaitEvent");
        replace(p.off, p.n, p.s, p.work);
        check_hip(hipEventRecord(ev_op, p.s), "hipEventRecord");
        last_replace = j;
    }

    // staggered: replace the pending sub-batches; st then follows the population's last operation
    void flush() {
        if (parts <= 1) return;
        while (!pending.empty()) replace_oldest();
        check_hip(hipStreamWaitEvent(st, ev_op, 0), "hipStreamWaitEvent");
    }

    // pop[k]'s fields, read behind the last replacement enqueued (staggered: the
    // pending half-batch stays pending, as ttga.ga.Island.snapshot)
    Member member_now(int k) {
        const hipStream_t s = parts > 1 ? part[last_replace].s : st;
        Member m{};
        uint8_t f = 0;
        check_hip(hipMemcpyAsync(&f, pop.feasible + k, 1, hipMemcpyDeviceToHost, s), "hipMemcpy");
        check_hip(hipMemcpyAsync(&m.scv, pop.scv + k, 4, hipMemcpyDeviceToHost, s), "hipMemcpy");
        check_hip(hipMemcpyAsync(&m.hcv, pop.hcv + k, 4, hipMemcpyDeviceToHost, s), "hipMemcpy");
        check_hip(hipMemcpyAsync(&m.penalty, pop.penalty + k, 4, hipMemcpyDeviceToHost, s), "hipMemcpy");
        check_hip(hipStreamSynchronize(s), "hipStreamSynchronize");
        m.feasible = f != 0;
        return m;
    }

    // pop[k]'s fields with every half-batch replaced
    Member member(int k) {
        flush();
        return member_now(k);
    }

    // the reference thread whose replacement put pop[0] in place (ga.cpp:580-585):
    // child c of the last tt_ga_replace (the source position it leaves at
    // tt_ga_work_source_offset in its work buffer), else 0
    int best_thread(bool after_step) {
        if (!after_step) return 0;
        const hipStream_t s = parts > 1 ? part[last_replace].s : st;
        const void* w = parts > 1 ? part[last_replace].work : work;
        const int base = parts > 1 ? part[last_replace].off : 0, nb = parts > 1 ? part[last_replace].n : C;
        int32_t src = 0;
        check_hip(hipMemcpyAsync(&src, (const uint8_t*)w + tt_ga_work_source_offset(N, E), 4, hipMemcpyDeviceToHost, s),
                  "hipMemcpy");
        check_hip(hipStreamSynchronize(s), "hipStreamSynchronize");
        const long k = N - nb;
        return src >= k && src < N ? (int)(base + src - k) : 0;
    }

    // setCurrentCost (ga.cpp:203-228) on pop[0] as the last replacement left it
    void log_cost(Output& out, std::chrono::steady_clock::time_point t0, int thread) {
        const Member m = member_now(0);
        long entry = 0;
        if (cost.offer(m.feasible, m.scv, m.hcv, entry)) out.line(log_line(entry, id, thread, seconds_since(t0)));
    }

    // serializeSolutions(k, 1, ...) (ga.cpp:318-342) into send_buf
    void pack(int k, uint8_t* send_buf) {
        auto cp = [&](void* dst, const void* src, size_t n) {
            check_hip(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
        };
        cp(send_buf, pop.slot + (size_t)k * E, E);
        cp(send_buf + E, pop.room + (size_t)k * E, E);
        cp(send_buf + 2 * E, pop.hcv + k, 4);
        cp(send_buf + 2 * E + 4, pop.scv + k, 4);
        cp(send_buf + 2 * E + 8, pop.penalty + k, 4);
        cp(send_buf + 2 * E + 12, pop.feasible + k, 1);
    }

    // deserializeSolution into position pos (ga.cpp:344-368)
    void unpack(int pos, const uint8_t* buf) {
        auto cp = [&](void* dst, const void* src, size_t n) {
            check_hip(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, st), "hipMemcpyAsync");
        };
        cp(pop.slot + (size_t)pos * E, buf, E);
        cp(pop.room + (size_t)pos * E, buf + E, E);
        cp(pop.hcv + pos, buf + 2 * E, 4);
        cp(pop.scv + pos, buf + 2 * E + 4, 4);
        cp(pop.penalty + pos, buf + 2 * E + 8, 4);
        cp(pop.feasible + pos, buf + 2 * E + 12, 1);
        if (parts > 1) check_hip(hipEventRecord(ev_op, st), "hipEventRecord");   // the next breed sees the migrants
    }

    void release() {
        pop.release();
        child.release();
        for (void* p : {(void*)rng_init, (void*)rng_child, (void*)flags, work, (void*)order, (void*)send_best,
                        (void*)send_second, (void*)recv_buf})
            if (p) (void)hipFree(p);
        for (size_t j = 1; j < part.size(); j++) {
            if (part[j].work) (void)hipFree(part[j].work);
            if (part[j].s) (void)hipStreamDestroy(part[j].s);
        }
        if (ev_op) (void)hipEventDestroy(ev_op);
        if (st) (void)hipStreamDestroy(st);
        if (tp) tt_problem_destroy(tp);
    }
};

// Reusable barrier for the island threads (the MPI_Barrier calls of ga.cpp:520,538).
class Barrier {
public:
    explicit Barrier(int n) : n_(n) {}
    void wait() {
        std::unique_lock<std::mutex> lk(mu_);
        const long gen = gen_;
        if (++count_ == n_) { count_ = 0; gen_++; cv_.notify_all(); return; }
        cv_.wait(lk, [&] { return gen != gen_; });
    }
private:
    std::mutex mu_;
    std::condition_variable cv_;
    int n_, count_ = 0;
    long gen_ = 0;
};

}  // namespace

int main(int argc, char** argv) {
    const auto t_start = std::chrono::steady_clock::now();
    if (argc == 3 && !std::strcmp(argv[1], "--replay-log")) return replay_log(argv[2]);
    Control ctl = parse_control(argc, argv);
    Output out(std::cout);                       // ga.cpp:60: -o is parsed, output goes to cout
    const Instance inst = read_tim(ctl.input);

    int ndev = 0;
    check_hip(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    const int G = ctl.gpus;
    if (G < 1 || G > ndev) die("--gpus " + std::to_string(G) + " but " + std::to_string(ndev) + " GPU(s) visible");
    const int K = ctl.islands > 0 ? ctl.islands : G;
    if (ctl.pop < 3) die("--pop must be at least 3 (ring migration writes pop[N-1] and pop[N-2])");
    const int N = ctl.pop;
    const int C = std::max(1, std::min(ctl.threads, N));
    const int gens = ctl.generations >= 0 ? ctl.generations : (2001 + C - 1) / C;   // generations 0..2000 (ga.cpp:510)
    if (ctl.rccl && K != G) die("--rccl needs one island per GPU (--islands equal to --gpus)");
    const bool rccl = K == G && (K > 1 || ctl.rccl);   // one island per GPU: RCCL ring; otherwise device copies

    std::vector<Island> isl(K);
    for (int k = 0; k < K; k++) {
        Island& I = isl[k];
        I.id = k; I.device = k % G; I.N = N; I.C = C;
        I.max_steps = max_steps_for(ctl.problem_type);
        I.seed = island_seed(ctl.seed, k);
        I.p1 = ctl.p1; I.p2 = ctl.p2; I.p3 = ctl.p3;
        I.parts = ctl.stagger >= 2 ? std::min(ctl.stagger, C) : 1;
    }
    std::vector<ncclComm_t> comms(K, nullptr);
    if (rccl) {
        std::vector<int> devs(K);
        for (int k = 0; k < K; k++) devs[k] = k;
        check_nccl(ncclCommInitAll(comms.data(), K, devs.data()), "ncclCommInitAll");
    }
    Barrier barrier(K);
    std::vector<long> best_value(K, 0);
    std::vector<int> best_feasible(K, 0);
    std::chrono::steady_clock::time_point t_begin;

    auto sync = [](Island& I) { check_hip(hipStreamSynchronize(I.st), "hipStreamSynchronize"); };
    auto run = [&](int k) {
        Island& I = isl[k];
        I.setup(inst);
        if (k == 0) I.initialize();
        sync(I);
        barrier.wait();
        // every island starts from island 0's population (ga.cpp:442-464)
        if (rccl) {
            check_nccl(ncclGroupStart(), "ncclGroupStart");
            check_nccl(ncclBroadcast(I.pop.slot, I.pop.slot, (size_t)N * I.E, ncclUint8, 0, comms[k], I.st), "bcast");
            check_nccl(ncclBroadcast(I.pop.room, I.pop.room, (size_t)N * I.E, ncclUint8, 0, comms[k], I.st), "bcast");
            check_nccl(ncclBroadcast(I.pop.hcv, I.pop.hcv, N, ncclInt32, 0, comms[k], I.st), "bcast");
            check_nccl(ncclBroadcast(I.pop.scv, I.pop.scv, N, ncclInt32, 0, comms[k], I.st), "bcast");
            check_nccl(ncclBroadcast(I.pop.penalty, I.pop.penalty, N, ncclInt32, 0, comms[k], I.st), "bcast");
            check_nccl(ncclBroadcast(I.pop.feasible, I.pop.feasible, N, ncclUint8, 0, comms[k], I.st), "bcast");
            check_nccl(ncclGroupEnd(), "ncclGroupEnd");
        } else if (k > 0) {
            const Pop& z = isl[0].pop;
            auto cp = [&](void* dst, const void* src, size_t n) {
                check_hip(hipMemcpyPeerAsync(dst, I.device, src, isl[0].device, n, I.st), "hipMemcpyPeerAsync");
            };
            cp(I.pop.slot, z.slot, (size_t)N * I.E);
            cp(I.pop.room, z.room, (size_t)N * I.E);
            cp(I.pop.hcv, z.hcv, 4 * (size_t)N);
            cp(I.pop.scv, z.scv, 4 * (size_t)N);
            cp(I.pop.penalty, z.penalty, 4 * (size_t)N);
            cp(I.pop.feasible, z.feasible, (size_t)N);
        }
        if (I.parts > 1) check_hip(hipEventRecord(I.ev_op, I.st), "hipEventRecord");   // the shared population
        sync(I);
        barrier.wait();
        if (k == 0) t_begin = std::chrono::steady_clock::now();      // beginTry (ga.cpp:476)
        barrier.wait();
        I.log_cost(out, t_begin, 0);
        const int right = (k + 1) % K, left = (k + K - 1) % K;
        for (int g = 0; g < gens; g++) {
            if ((g + 1) % 100 == 50) {   // ga.cpp:514-540, one migrant each way
                I.flush();                                // staggered: the pending sub-batches replaced first
                I.pack(0, I.send_best);                   // best, then 2nd best (N >= 3: untouched by dir 0)
                I.pack(1, I.send_second);
                sync(I);
                barrier.wait();
                uint8_t* from_left = I.recv_buf;          // dir 0: left's best -> pop[N-1]
                uint8_t* from_right = I.recv_buf + I.migrant_bytes;   // dir 1: right's 2nd best -> pop[N-2]
                if (rccl) {
                    check_nccl(ncclGroupStart(), "ncclGroupStart");
                    check_nccl(ncclSend(I.send_best, I.migrant_bytes, ncclUint8, right, comms[k], I.st), "ncclSend");
                    check_nccl(ncclRecv(from_left, I.migrant_bytes, ncclUint8, left, comms[k], I.st), "ncclRecv");
                    check_nccl(ncclGroupEnd(), "ncclGroupEnd");
                    check_nccl(ncclGroupStart(), "ncclGroupStart");
                    check_nccl(ncclSend(I.send_second, I.migrant_bytes, ncclUint8, left, comms[k], I.st), "ncclSend");
                    check_nccl(ncclRecv(from_right, I.migrant_bytes, ncclUint8, right, comms[k], I.st), "ncclRecv");
                    check_nccl(ncclGroupEnd(), "ncclGroupEnd");
                } else {
                    check_hip(hipMemcpyPeerAsync(from_left, I.device, isl[left].send_best, isl[left].device,
                                                 I.migrant_bytes, I.st), "hipMemcpyPeerAsync");
                    check_hip(hipMemcpyPeerAsync(from_right, I.device, isl[right].send_second, isl[right].device,
                                                 I.migrant_bytes, I.st), "hipMemcpyPeerAsync");
                }
                I.unpack(N - 1, from_left);
                I.unpack(N - 2, from_right);
                sync(I);
                barrier.wait();      // the neighbours' send buffers are free again
            }
            I.step();
            I.log_cost(out, t_begin, I.best_thread(true));
        }
        const Member b = I.member(0);
        best_feasible[k] = b.feasible;
        best_value[k] = b.feasible ? b.scv : (long)b.hcv * 1000000 + b.scv;
    };
    std::vector<std::thread> th;
    for (int k = 0; k < K; k++) th.emplace_back(run, k);
    for (auto& t : th) t.join();

    // setGlobalCost (ga.cpp:234-257): MIN over islands (RCCL all-reduce across GPUs), printed once
    long gmin = *std::min_element(best_value.begin(), best_value.end());
    if (rccl) {
        std::vector<std::thread> red;
        std::vector<int64_t*> dv(K, nullptr);        // hcv * 1e6 + scv can pass 2^31
        for (int k = 0; k < K; k++)
            red.emplace_back([&, k] {
                Island& I = isl[k];
                check_hip(hipSetDevice(I.device), "hipSetDevice");
                check_hip(hipMalloc(&dv[k], 8), "hipMalloc");
                const int64_t v = best_value[k];
                check_hip(hipMemcpy(dv[k], &v, 8, hipMemcpyHostToDevice), "hipMemcpy");
                check_nccl(ncclAllReduce(dv[k], dv[k], 1, ncclInt64, ncclMin, comms[k], I.st), "ncclAllReduce");
                check_hip(hipStreamSynchronize(I.st), "hipStreamSynchronize");
            });
        for (auto& t : red) t.join();
        int64_t v = 0;
        check_hip(hipSetDevice(0), "hipSetDevice");
        check_hip(hipMemcpy(&v, dv[0], 8, hipMemcpyDeviceToHost), "hipMemcpy");
        gmin = v;
        for (int k = 0; k < K; k++) { (void)hipSetDevice(k); (void)hipFree(dv[k]); }
    }
    out.line(run_best_line(best_feasible[0] != 0, gmin));
    // endTry (ga.cpp:169-197) per island
    for (int k = 0; k < K; k++) {
        Island& I = isl[k];
        check_hip(hipSetDevice(I.device), "hipSetDevice");
        const Member b = I.member(0);
        std::vector<uint8_t> sl(I.E), rm(I.E);
        check_hip(hipMemcpy(sl.data(), I.pop.slot, I.E, hipMemcpyDeviceToHost), "hipMemcpy");
        check_hip(hipMemcpy(rm.data(), I.pop.room, I.E, hipMemcpyDeviceToHost), "hipMemcpy");
        out.line(solution_line(b.feasible, b.scv, b.hcv, sl, rm, k, seconds_since(t_begin)));
    }
    out.line(run_final_line(K, C, seconds_since(t_start)));
    for (int k = 0; k < K; k++) {
        (void)hipSetDevice(isl[k].device);
        isl[k].release();
        if (comms[k]) ncclCommDestroy(comms[k]);
    }
    return 0;
}

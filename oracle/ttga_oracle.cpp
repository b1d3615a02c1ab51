// ttga oracle — TEST INFRASTRUCTURE ONLY (the checker, never the product path).
//
// A clean-room CPU restatement of the reference's hot-path arithmetic
// (nelilepo/timetabling-ga-mpi-openmp, reference tree at /root/reference).
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
// load the shared library built from this file (oracle/libttoracle.so).
//
// Parity is PINNED: this restatement is checked bit-for-bit against golden
// vectors produced by the reference's own Problem.cpp / Solution.cpp /
// Random.cc compiled unmodified (oracle/ref_harness.cpp, oracle/Makefile,
// F1 convention via -ftrivial-auto-var-init=zero), see tests/golden/.
//
// It deliberately keeps the reference's data structures and loop order
// (per-slot ascending event lists, int32 row-major matrices, per-student
// scans) so that it doubles as the "port" CPU baseline. Each function cites
// the reference lines it restates.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

const int kSlots = 45;      // 5 days x 9 slots, Solution.cpp:52,57,94,100
const int kSlotsPerDay = 9;

// Park-Miller minimal standard generator with Schrage's method.
// Random.h:15-19 (IA, IM, AM, IQ, IR), Random.cc:27-37 (ran01).
inline double pm_next(long* s) {
    const long IA = 16807, IM = 2147483647, IQ = 127773, IR = 2836;
    const double AM = 1.0 / IM;
    long k = (*s) / IQ;
    *s = IA * (*s - k * IQ) - IR * k;
    if (*s < 0) *s += IM;
    return AM * (*s);
}

struct Problem {
    int E, R, F, S;
    std::vector<int> room_size;       // R                 Problem.h:40
    std::vector<int> A;               // S x E (row-major) Problem.h:41
    std::vector<int> room_feat;       // R x F             Problem.h:43
    std::vector<int> event_feat;      // E x F             Problem.h:44
    std::vector<int> student_number;  // E                 Problem.h:39
    std::vector<int> corr;            // E x E             Problem.h:42
    std::vector<int> possible;        // E x R             Problem.h:46
    int a(int s, int e) const { return A[(size_t)s * E + e]; }
    int c(int i, int j) const { return corr[(size_t)i * E + j]; }
    int p(int e, int r) const { return possible[(size_t)e * R + r]; }
};

// Derived matrices, Problem.cpp:33-95.
void derive(Problem& P) {
    const int E = P.E, R = P.R, F = P.F, S = P.S;
    P.student_number.assign(E, 0);
    for (int i = 0; i < E; i++) {                       // Problem.cpp:33-40
        int sum = 0;
        for (int j = 0; j < S; j++) sum += P.a(j, i);
        P.student_number[i] = sum;
    }
    // Problem.cpp:42-58: corr[i][j] = 1 iff some student k has A[k][i]==1 and
    // A[k][j]==1 (diagonal included). Restated student-major (same set, the
    // E*E*S triple loop is 108 s at E=2000,S=5000): for each student, mark
    // every ordered pair of the events it attends.
    P.corr.assign((size_t)E * E, 0);
    std::vector<int> ev;
    for (int k = 0; k < S; k++) {
        ev.clear();
        for (int e = 0; e < E; e++)
            if (P.a(k, e) == 1) ev.push_back(e);
        for (size_t x = 0; x < ev.size(); x++)
            for (size_t y = 0; y < ev.size(); y++) P.corr[(size_t)ev[x] * E + ev[y]] = 1;
    }
    P.possible.assign((size_t)E * R, 0);                // Problem.cpp:76-95
    for (int i = 0; i < E; i++) {
        for (int j = 0; j < R; j++) {
            if (P.room_size[j] >= P.student_number[i]) {
                int k;
                for (k = 0; k < F; k++)
                    if (P.event_feat[(size_t)i * F + k] == 1 && P.room_feat[(size_t)j * F + k] == 0) break;
                if (k == F) P.possible[(size_t)i * R + j] = 1;
            }
        }
    }
}

// One individual: Solution.h:36-37 (sln pairs + timeslot_events map).
struct Sol {
    std::vector<int> slot, room;
    std::vector<std::vector<int> > lists;  // lists[t]: events in slot t, ascending
    Sol() : lists(kSlots) {}
};

void build_lists(Sol& s) {
    for (int t = 0; t < kSlots; t++) s.lists[t].clear();
    for (size_t e = 0; e < s.slot.size(); e++) s.lists[s.slot[e]].push_back((int)e);
}

// ---------------------------------------------------------------- evaluation
// Solution.cpp:63-84
bool compute_feasibility(const Problem& P, const Sol& s) {
    const int E = P.E;
    for (int i = 0; i < E; i++) {
        for (int j = i + 1; j < E; j++) {
            if (s.slot[i] == s.slot[j] && s.room[i] == s.room[j]) return false;
            if (P.c(i, j) == 1 && s.slot[i] == s.slot[j]) return false;
        }
        if (P.p(i, s.room[i]) == 0) return false;
    }
    return true;
}

// Solution.cpp:86-139
int compute_scv(const Problem& P, const Sol& s) {
    int scv = 0;
    for (int i = 0; i < P.E; i++)
        if (s.slot[i] % kSlotsPerDay == 8) scv += P.student_number[i];
    for (int j = 0; j < P.S; j++) {
        int consecutive = 0;
        for (int i = 0; i < kSlots; i++) {
            if (i % kSlotsPerDay == 0) consecutive = 0;
            bool attends = false;
            const std::vector<int>& L = s.lists[i];
            for (size_t k = 0; k < L.size(); k++) {
                if (P.a(j, L[k]) == 1) {
                    attends = true;
                    consecutive++;
                    if (consecutive > 2) scv++;
                    break;
                }
            }
            if (!attends) consecutive = 0;
        }
    }
    for (int j = 0; j < P.S; j++) {
        for (int d = 0; d < 5; d++) {
            int classes = 0;
            for (int t = 0; t < kSlotsPerDay; t++) {
                const std::vector<int>& L = s.lists[kSlotsPerDay * d + t];
                for (size_t k = 0; k < L.size(); k++) {
                    if (P.a(j, L[k]) == 1) { classes++; break; }
                }
                if (classes > 1) break;
            }
            if (classes == 1) scv++;
        }
    }
    return scv;
}

// Solution.cpp:141-160
int compute_hcv(const Problem& P, const Sol& s) {
    int hcv = 0;
    for (int i = 0; i < P.E; i++) {
        for (int j = i + 1; j < P.E; j++) {
            if (s.slot[i] == s.slot[j] && s.room[i] == s.room[j]) hcv++;
            if (s.slot[i] == s.slot[j] && P.c(i, j) == 1) hcv++;
        }
        if (P.p(i, s.room[i]) == 0) hcv++;
    }
    return hcv;
}

// ------------------------------------------------------------ room matching
// Solution.cpp:852-891 (networkFlow), literal dense-matrix restatement.
struct Flow {
    int V;
    std::vector<int> size, flow, val, dad;
    int& sz(int i, int j) { return size[(size_t)i * (V + 1) + j]; }
    int& fl(int i, int j) { return flow[(size_t)i * (V + 1) + j]; }
};

bool network_flow(Flow& g) {
    const int V = g.V;
    g.val.assign(V + 1, -10);
    g.dad.assign(V + 1, 0);
    g.val[0] = -11;
    g.val[1] = -9;
    int k, t, mn = 0;
    for (k = 1; k != 0; k = mn, mn = 0) {
        g.val[k] = 10 + g.val[k];
        if (g.val[k] == 0) return false;
        if (k == V) return true;
        for (t = 1; t <= V; t++) {
            if (g.val[t] < 0) {
                int pr = -g.fl(k, t);
                if (g.sz(k, t) > 0) pr += g.sz(k, t);
                if (pr > g.val[k]) pr = g.val[k];
                pr = 10 - pr;
                if (g.sz(k, t) && g.val[t] < -pr) {
                    g.val[t] = -pr;
                    g.dad[t] = k;
                }
                if (g.val[t] > g.val[mn]) mn = t;
            }
        }
    }
    return false;
}

// Solution.cpp:836-849 (maxMatching)
void max_matching(Flow& g) {
    const int V = g.V;
    while (network_flow(g)) {
        int x = g.dad[V], y = V;
        while (x != 0) {
            g.fl(x, y) = g.fl(x, y) + g.val[V];
            g.fl(y, x) = -g.fl(x, y);
            y = x;
            x = g.dad[y];
        }
    }
}

// Solution.cpp:772-833 (assignRooms) with busy[] zero-initialised.
void assign_rooms(const Problem& P, Sol& s, int t) {
    const std::vector<int>& L = s.lists[t];
    const int N = (int)L.size(), R = P.R;
    Flow g;
    g.V = N + 2 + R;
    const int V = g.V;
    g.size.assign((size_t)(V + 1) * (V + 1), 0);
    g.flow.assign((size_t)(V + 1) * (V + 1), 0);
    for (int i = 0; i < N; i++) {
        g.sz(1, i + 2) = 1;
        g.sz(i + 2, 1) = -1;
        for (int j = 0; j < R; j++)
            if (P.p(L[i], j) == 1) {
                g.sz(i + 2, N + j + 2) = 1;
                g.sz(N + j + 2, i + 2) = -1;
                g.sz(N + j + 2, V) = 1;
                g.sz(V, N + j + 2) = -1;
            }
    }
    max_matching(g);
    std::vector<int> busy(R, 0), assigned(N, 0);
    int less_busy = 0;                    // declared once per call (Solution.cpp:777)
    for (int i = 0; i < N; i++) {
        for (int j = 0; j < R; j++) {
            if (g.fl(i + 2, N + j + 2) == 1) {
                s.room[L[i]] = j;
                assigned[i] = 1;
                busy[j] += 1;
            }
        }
    }
    for (int i = 0; i < N; i++) {
        if (assigned[i] == 0) {
            for (int j = 0; j < R; j++)
                if (P.p(L[i], j) == 1) { less_busy = j; break; }
            for (int j = 0; j < R; j++)
                if (P.p(L[i], j) == 1 && busy[j] < busy[less_busy]) less_busy = j;
            s.room[L[i]] = less_busy;
        }
    }
}

void assign_all(const Problem& P, Sol& s) {
    for (int t = 0; t < kSlots; t++)
        if (!s.lists[t].empty()) assign_rooms(P, s, t);
}

// -------------------------------------------------------------------- moves
void erase_one(std::vector<int>& L, int e) {
    std::vector<int>::iterator it = std::find(L.begin(), L.end(), e);
    if (it != L.end()) L.erase(it);
}

// Solution.cpp:357-376
void move1(const Problem& P, Sol& s, int e, int t) {
    int ts = s.slot[e];
    s.slot[e] = t;
    erase_one(s.lists[ts], e);
    s.lists[t].push_back(e);
    std::sort(s.lists[t].begin(), s.lists[t].end());
    assign_rooms(P, s, t);
    if (!s.lists[ts].empty()) assign_rooms(P, s, ts);
}

// Solution.cpp:378-403
void move2(const Problem& P, Sol& s, int e1, int e2) {
    int t = s.slot[e1];
    s.slot[e1] = s.slot[e2];
    s.slot[e2] = t;
    erase_one(s.lists[t], e1);
    s.lists[t].push_back(e2);
    erase_one(s.lists[s.slot[e1]], e2);
    s.lists[s.slot[e1]].push_back(e1);
    std::sort(s.lists[t].begin(), s.lists[t].end());
    std::sort(s.lists[s.slot[e1]].begin(), s.lists[s.slot[e1]].end());
    assign_rooms(P, s, s.slot[e1]);
    assign_rooms(P, s, s.slot[e2]);
}

// Solution.cpp:405-439
void move3(const Problem& P, Sol& s, int e1, int e2, int e3) {
    int t = s.slot[e1];
    s.slot[e1] = s.slot[e2];
    s.slot[e2] = s.slot[e3];
    s.slot[e3] = t;
    erase_one(s.lists[t], e1);
    s.lists[t].push_back(e3);
    erase_one(s.lists[s.slot[e1]], e2);
    s.lists[s.slot[e1]].push_back(e1);
    erase_one(s.lists[s.slot[e2]], e3);
    s.lists[s.slot[e2]].push_back(e2);
    std::sort(s.lists[s.slot[e1]].begin(), s.lists[s.slot[e1]].end());
    std::sort(s.lists[s.slot[e2]].begin(), s.lists[s.slot[e2]].end());
    std::sort(s.lists[s.slot[e3]].begin(), s.lists[s.slot[e3]].end());
    assign_rooms(P, s, s.slot[e1]);
    assign_rooms(P, s, s.slot[e2]);
    assign_rooms(P, s, s.slot[e3]);
}

// Solution.cpp:441-469
void random_move(const Problem& P, Sol& s, long* rng) {
    const int E = P.E;
    int type = (int)(pm_next(rng) * 3) + 1;
    int e1 = (int)(pm_next(rng) * E);
    if (type == 1) {
        int t = (int)(pm_next(rng) * 45);
        move1(P, s, e1, t);
    } else if (type == 2) {
        int e2 = (int)(pm_next(rng) * E);
        while (e2 == e1) e2 = (int)(pm_next(rng) * E);
        move2(P, s, e1, e2);
    } else {
        int e2 = (int)(pm_next(rng) * E);
        while (e2 == e1) e2 = (int)(pm_next(rng) * E);
        int e3 = (int)(pm_next(rng) * E);
        while (e3 == e1 || e3 == e2) e3 = (int)(pm_next(rng) * E);
        move3(P, s, e1, e2, e3);
    }
}

// ------------------------------------------------------------ delta evals
// Solution.cpp:173-191
int event_hcv(const Problem& P, const Sol& s, int e) {
    int h = 0;
    const std::vector<int>& L = s.lists[s.slot[e]];
    for (size_t i = 0; i < L.size(); i++) {
        if (L[i] != e) {
            if (s.room[e] == s.room[L[i]]) h++;
            if (P.c(e, L[i]) == 1) h++;
        }
    }
    return h;
}

// Solution.cpp:194-215
int event_affected_hcv(const Problem& P, const Sol& s, int e) {
    int h = 0;
    const std::vector<int>& L = s.lists[s.slot[e]];
    for (size_t i = 0; i < L.size(); i++) {
        for (size_t j = i + 1; j < L.size(); j++)
            if (s.room[L[i]] == s.room[L[j]]) h++;
        if (L[i] != e && P.c(e, L[i]) == 1) h++;
    }
    return h;
}

// Solution.cpp:235-245
int affected_room_in_timeslot_hcv(const Sol& s, int t) {
    int h = 0;
    const std::vector<int>& L = s.lists[t];
    for (size_t i = 0; i < L.size(); i++)
        for (size_t j = i + 1; j < L.size(); j++)
            if (s.room[L[i]] == s.room[L[j]]) h++;
    return h;
}

bool attends_slot(const Problem& P, const Sol& s, int student, int t) {
    const std::vector<int>& L = s.lists[t];
    for (size_t k = 0; k < L.size(); k++)
        if (P.a(student, L[k]) == 1) return true;
    return false;
}

// Solution.cpp:248-324
int event_scv(const Problem& P, const Sol& s, int e) {
    int scv = 0;
    const int t = s.slot[e];
    int single = P.student_number[e];
    if (t % 9 == 8) scv += P.student_number[e];
    for (int i = 0; i < P.S; i++) {
        if (P.a(i, e) != 1) continue;
        if (t % 9 < 8) {
            // first event of slot t+1 the student attends decides (Solution.cpp:262-286)
            bool found = false;
            const std::vector<int>& L1 = s.lists[t + 1];
            for (size_t j = 0; j < L1.size(); j++) {
                if (P.a(i, L1[j]) == 1) {
                    if (t % 9 < 7 && attends_slot(P, s, i, t + 2)) { scv++; found = true; }
                    if (t % 9 > 0 && attends_slot(P, s, i, t - 1)) { scv++; found = true; }
                }
                if (found) break;
            }
        }
        if (t % 9 > 1) {                                  // Solution.cpp:288-301
            if (attends_slot(P, s, i, t - 1) && attends_slot(P, s, i, t - 2)) scv++;
        }
        for (int d = t - (t % 9); d < t - (t % 9) + 9; d++) {  // Solution.cpp:303-317
            if (d != t && attends_slot(P, s, i, d)) { single--; break; }
        }
    }
    return scv + single;
}

// Solution.cpp:329-355
int single_classes_scv(const Problem& P, const Sol& s, int e) {
    const int t = s.slot[e];
    int single = 0;
    for (int i = 0; i < P.S; i++) {
        if (P.a(i, e) != 1) continue;
        int classes = 0;
        for (int d = t - (t % 9); d < t - (t % 9) + 9; d++) {
            if (classes > 1) break;
            if (d != t && attends_slot(P, s, i, d)) classes++;
        }
        if (classes == 1) single++;
    }
    return single;
}

// ------------------------------------------------------------ local search
// Solution.cpp:471-769 (LS_limit never binds at its 999999 s default, the
// timer checks are therefore omitted; step budget shared by both phases).
void local_search(const Problem& P, Sol& s, long* rng, int max_steps, double p1, double p2, double p3) {
    const int E = P.E;
    std::vector<int> ev(E);
    for (int i = 0; i < E; i++) ev[i] = i;
    for (int i = 0; i < E; i++) {                       // Solution.cpp:479-484
        int j = (int)(pm_next(rng) * E);
        int h = ev[i]; ev[i] = ev[j]; ev[j] = h;
    }
    int step = 0;
    bool better = false;
    int evc = 0;
    Sol nb;
    if (!compute_feasibility(P, s)) {                   // phase 1, Solution.cpp:497-618
        for (int i = 0; evc < E; i = (i + 1) % E) {
            if (step > max_steps) break;
            const int ei = ev[i];
            if (event_hcv(P, s, ei) == 0) { evc++; continue; }
            int t_start = (int)(pm_next(rng) * 45);
            int t_orig = s.slot[ei];
            for (int h = 0, t = t_start; h < 45; t = (t + 1) % 45, h++) {
                if (step > max_steps) break;
                if (pm_next(rng) < p1) {
                    step++;
                    nb = s;
                    move1(P, nb, ei, t);
                    int n = event_affected_hcv(P, nb, ei) + affected_room_in_timeslot_hcv(nb, t_orig);
                    int c = event_affected_hcv(P, s, ei) + affected_room_in_timeslot_hcv(s, t);
                    if (n < c) { s = nb; evc = 0; better = true; break; }
                }
            }
            if (better) { better = false; continue; }
            if (p2 != 0) {
                for (int j = (i + 1) % E; j != i; j = (j + 1) % E) {
                    if (step > max_steps) break;
                    if (pm_next(rng) < p2) {
                        step++;
                        const int ej = ev[j];
                        nb = s;
                        move2(P, nb, ei, ej);
                        int n = event_affected_hcv(P, nb, ei) + event_affected_hcv(P, nb, ej);
                        int c = event_affected_hcv(P, s, ei) + event_affected_hcv(P, s, ej);
                        if (n < c) { s = nb; evc = 0; better = true; break; }
                    }
                }
                if (better) { better = false; continue; }
            }
            if (p3 != 0) {
                for (int j = (i + 1) % E; j != i; j = (j + 1) % E) {
                    if (step > max_steps) break;
                    for (int k = (j + 1) % E; k != i; k = (k + 1) % E) {
                        if (step > max_steps) break;
                        const int ej = ev[j], ek = ev[k];
                        if (pm_next(rng) < p3) {
                            step++;
                            int c = event_affected_hcv(P, s, ei) + event_affected_hcv(P, s, ej) + event_affected_hcv(P, s, ek);
                            nb = s;
                            move3(P, nb, ei, ej, ek);
                            int n = event_affected_hcv(P, nb, ei) + event_affected_hcv(P, nb, ej) + event_affected_hcv(P, nb, ek);
                            if (n < c) { s = nb; evc = 0; better = true; break; }
                        }
                        if (step > max_steps) break;
                        if (pm_next(rng) < p3) {
                            step++;
                            int c = event_affected_hcv(P, s, ei) + event_affected_hcv(P, s, ek) + event_affected_hcv(P, s, ej);
                            nb = s;
                            move3(P, nb, ei, ek, ej);
                            int n = event_affected_hcv(P, nb, ei) + event_affected_hcv(P, nb, ek) + event_affected_hcv(P, nb, ej);
                            if (n < c) { s = nb; evc = 0; better = true; break; }
                        }
                    }
                    if (better) break;
                }
                if (better) { better = false; continue; }
            }
            evc++;
        }
    }
    if (compute_feasibility(P, s)) {                    // phase 2, Solution.cpp:619-768
        evc = 0;
        for (int i = 0; evc < E; i = (i + 1) % E) {
            if (step > max_steps) break;
            const int ei = ev[i];
            int cur = event_scv(P, s, ei);
            if (cur == 0) { evc++; continue; }
            int t_start = (int)(pm_next(rng) * 45);
            for (int h = 0, t = t_start; h < 45; t = (t + 1) % 45, h++) {
                if (step > max_steps) break;
                if (pm_next(rng) < p1) {
                    step++;
                    nb = s;
                    move1(P, nb, ei, t);
                    if (event_affected_hcv(P, nb, ei) == 0) {
                        int n = event_scv(P, nb, ei) + single_classes_scv(P, s, ei) - single_classes_scv(P, nb, ei);
                        if (n < cur) { s = nb; evc = 0; better = true; break; }
                    }
                }
            }
            if (better) { better = false; continue; }
            if (p2 != 0) {
                for (int j = (i + 1) % E; j != i; j = (j + 1) % E) {
                    if (step > max_steps) break;
                    if (pm_next(rng) < p2) {
                        step++;
                        const int ej = ev[j];
                        nb = s;
                        move2(P, nb, ei, ej);
                        if (event_affected_hcv(P, nb, ei) + event_affected_hcv(P, nb, ej) == 0) {
                            int n = event_scv(P, nb, ei) + single_classes_scv(P, s, ei) - single_classes_scv(P, nb, ei)
                                  + event_scv(P, nb, ej) + single_classes_scv(P, s, ej) - single_classes_scv(P, nb, ej);
                            if (n < cur + event_scv(P, s, ej)) { s = nb; evc = 0; better = true; break; }
                        }
                    }
                }
                if (better) { better = false; continue; }
            }
            if (p3 != 0) {
                for (int j = (i + 1) % E; j != i; j = (j + 1) % E) {
                    if (step > max_steps) break;
                    for (int k = (j + 1) % E; k != i; k = (k + 1) % E) {
                        if (step > max_steps) break;
                        const int ej = ev[j], ek = ev[k];
                        if (pm_next(rng) < p3) {
                            step++;
                            nb = s;
                            move3(P, nb, ei, ej, ek);
                            if (event_affected_hcv(P, nb, ei) + event_affected_hcv(P, nb, ej) + event_affected_hcv(P, nb, ek) == 0) {
                                int n = event_scv(P, nb, ei) + single_classes_scv(P, s, ei) - single_classes_scv(P, nb, ei)
                                      + event_scv(P, nb, ej) + single_classes_scv(P, s, ej) - single_classes_scv(P, nb, ej)
                                      + event_scv(P, nb, ek) + single_classes_scv(P, s, ek) - single_classes_scv(P, nb, ek);
                                if (n < cur + event_scv(P, s, ej) + event_scv(P, s, ek)) { s = nb; evc = 0; better = true; break; }
                            }
                        }
                        if (step > max_steps) break;
                        if (pm_next(rng) < p3) {
                            step++;
                            nb = s;
                            move3(P, nb, ei, ek, ej);
                            if (event_affected_hcv(P, nb, ei) + event_affected_hcv(P, nb, ek) + event_affected_hcv(P, nb, ej) == 0) {
                                int n = event_scv(P, nb, ei) + single_classes_scv(P, s, ei) - single_classes_scv(P, nb, ei)
                                      + event_scv(P, nb, ek) + single_classes_scv(P, s, ek) - single_classes_scv(P, nb, ek)
                                      + event_scv(P, nb, ej) + single_classes_scv(P, s, ej) - single_classes_scv(P, nb, ej);
                                if (n < cur + event_scv(P, s, ek) + event_scv(P, s, ej)) { s = nb; evc = 0; better = true; break; }
                            }
                        }
                    }
                    if (better) break;
                }
                if (better) { better = false; continue; }
            }
            evc++;
        }
    }
}

void load(const Problem& P, Sol& s, const uint8_t* slot, const uint8_t* room) {
    s.slot.assign(slot, slot + P.E);
    if (room) s.room.assign(room, room + P.E);
    else s.room.assign(P.E, -1);
    build_lists(s);
}

void store(const Problem& P, const Sol& s, uint8_t* slot, uint8_t* room) {
    for (int e = 0; e < P.E; e++) {
        if (slot) slot[e] = (uint8_t)s.slot[e];
        if (room) room[e] = (uint8_t)s.room[e];
    }
}

}  // namespace

extern "C" {

// Problem(istream&) equivalent from already-parsed arrays (Problem.cpp:3-96).
void* tto_problem_create(int E, int R, int F, int S, const int* room_size, const int* A,
                         const int* room_feat, const int* event_feat) {
    Problem* P = new Problem();
    P->E = E; P->R = R; P->F = F; P->S = S;
    P->room_size.assign(room_size, room_size + R);
    P->A.assign(A, A + (size_t)S * E);
    P->room_feat.assign(room_feat, room_feat + (size_t)R * F);
    P->event_feat.assign(event_feat, event_feat + (size_t)E * F);
    derive(*P);
    return P;
}

void tto_problem_destroy(void* p) { delete (Problem*)p; }

void tto_problem_derived(const void* p, int* student_number, int* corr, int* possible) {
    const Problem& P = *(const Problem*)p;
    std::copy(P.student_number.begin(), P.student_number.end(), student_number);
    std::copy(P.corr.begin(), P.corr.end(), corr);
    std::copy(P.possible.begin(), P.possible.end(), possible);
}

// Random::next stream (Random.cc:27-37); writes n draws and the final state.
void tto_rand(long seed, int n, double* out, long* final_state) {
    long s = seed;
    for (int i = 0; i < n; i++) out[i] = pm_next(&s);
    *final_state = s;
}

// Batched computeFeasibility / computeHcv / computeScv / computePenalty
// (Solution.cpp:63-170). Population is individual-major: slot[P][E], room[P][E].
void tto_eval(const void* p, const uint8_t* slot, const uint8_t* room, int np, int32_t* hcv,
              int32_t* scv, uint8_t* feasible, int32_t* penalty) {
    const Problem& P = *(const Problem*)p;
    Sol s;
    for (int i = 0; i < np; i++) {
        load(P, s, slot + (size_t)i * P.E, room + (size_t)i * P.E);
        bool f = compute_feasibility(P, s);
        int h = compute_hcv(P, s);
        int c = compute_scv(P, s);
        hcv[i] = h;
        scv[i] = c;
        feasible[i] = f ? 1 : 0;
        penalty[i] = f ? c : 1000000 + h;   // Solution.cpp:162-170
    }
}

// assignRooms over every non-empty slot in ascending t (RandomInitialSolution order).
void tto_assign_rooms(const void* p, const uint8_t* slot, uint8_t* room, int np) {
    const Problem& P = *(const Problem*)p;
    Sol s;
    for (int i = 0; i < np; i++) {
        load(P, s, slot + (size_t)i * P.E, 0);
        assign_all(P, s);
        store(P, s, 0, room + (size_t)i * P.E);
    }
}

// Solution::RandomInitialSolution (Solution.cpp:48-61), one Random stream per individual.
void tto_random_init(const void* p, int64_t* rng, uint8_t* slot, uint8_t* room, int np) {
    const Problem& P = *(const Problem*)p;
    Sol s;
    for (int i = 0; i < np; i++) {
        long st = (long)rng[i];
        s.slot.assign(P.E, 0);
        s.room.assign(P.E, -1);
        for (int t = 0; t < kSlots; t++) s.lists[t].clear();
        for (int e = 0; e < P.E; e++) {
            int t = (int)(pm_next(&st) * 45);
            s.slot[e] = t;
            s.lists[t].push_back(e);
        }
        assign_all(P, s);
        store(P, s, slot + (size_t)i * P.E, room + (size_t)i * P.E);
        rng[i] = st;
    }
}

// Solution::localSearch (Solution.cpp:471-769), one Random stream per individual.
void tto_local_search(const void* p, uint8_t* slot, uint8_t* room, int64_t* rng, int np, int max_steps,
                      double p1, double p2, double p3) {
    const Problem& P = *(const Problem*)p;
    Sol s;
    for (int i = 0; i < np; i++) {
        load(P, s, slot + (size_t)i * P.E, room + (size_t)i * P.E);
        long st = (long)rng[i];
        local_search(P, s, &st, max_steps, p1, p2, p3);
        store(P, s, slot + (size_t)i * P.E, room + (size_t)i * P.E);
        rng[i] = st;
    }
}

// Solution::crossover on a fresh child (Solution.cpp:893-910 without the F2
// stale-list defect): per event next()<0.5 picks parent1's slot, then
// assignRooms on every non-empty slot.
void tto_crossover(const void* p, const uint8_t* slot1, const uint8_t* slot2, int64_t* rng, uint8_t* slot,
                   uint8_t* room, int np) {
    const Problem& P = *(const Problem*)p;
    Sol s;
    for (int i = 0; i < np; i++) {
        long st = (long)rng[i];
        s.slot.assign(P.E, 0);
        s.room.assign(P.E, -1);
        for (int e = 0; e < P.E; e++) {
            size_t off = (size_t)i * P.E + e;
            s.slot[e] = pm_next(&st) < 0.5 ? slot1[off] : slot2[off];
        }
        build_lists(s);
        assign_all(P, s);
        store(P, s, slot + (size_t)i * P.E, room + (size_t)i * P.E);
        rng[i] = st;
    }
}

// Solution::mutation -> randomMove (Solution.cpp:441-469,912-914), in place.
void tto_mutation(const void* p, uint8_t* slot, uint8_t* room, int64_t* rng, int np) {
    const Problem& P = *(const Problem*)p;
    Sol s;
    for (int i = 0; i < np; i++) {
        load(P, s, slot + (size_t)i * P.E, room + (size_t)i * P.E);
        long st = (long)rng[i];
        random_move(P, s, &st);
        store(P, s, slot + (size_t)i * P.E, room + (size_t)i * P.E);
        rng[i] = st;
    }
}

// GA generation primitives (the batched restatement of ga.cpp:543-585, see
// include/ttga.h tt_ga_breed / tt_ga_replace). Child c uses stream rng[c].
void tto_ga_breed(const void* p, const uint8_t* pop_slot, const uint8_t* pop_room, const int32_t* pen, int N,
                  int64_t* rng, int C, double p_cross, double p_mut, int skip_init, uint8_t* child_slot,
                  uint8_t* child_room, uint8_t* flags) {
    const Problem& P = *(const Problem*)p;
    const int E = P.E;
    Sol s;
    for (int c = 0; c < C; c++) {
        long st = (long)rng[c];
        if (skip_init)                                        // ga.cpp:543-548
            for (int k = 0; k < 3 * E; k++) pm_next(&st);
        int par[2];
        for (int q = 0; q < 2; q++) {                         // selection5, ga.cpp:129-145
            int best = (int)(pm_next(&st) * N);
            for (int i = 1; i < 5; i++) {
                int t = (int)(pm_next(&st) * N);
                if ((uint32_t)pen[t] < (uint32_t)pen[best]) best = t;   // invalid (-1) ranks last
            }
            par[q] = best;
        }
        uint8_t f = 0;
        const uint8_t* sa = pop_slot + (size_t)par[0] * E;
        const uint8_t* sb = pop_slot + (size_t)par[1] * E;
        if (pm_next(&st) < p_cross) {                         // ga.cpp:562-563
            f |= 1;
            s.slot.assign(E, 0);
            s.room.assign(E, -1);
            for (int e = 0; e < E; e++) s.slot[e] = pm_next(&st) < 0.5 ? sa[e] : sb[e];
            build_lists(s);
            assign_all(P, s);
        } else {                                              // ga.cpp:564-566
            load(P, s, sa, pop_room + (size_t)par[0] * E);
        }
        if (pm_next(&st) < p_mut) {                           // ga.cpp:569-571
            f |= 2;
            random_move(P, s, &st);
        }
        store(P, s, child_slot + (size_t)c * E, child_room + (size_t)c * E);
        flags[c] = f;
        rng[c] = st;
    }
}

// children overwrite positions N-C..N-1 (ga.cpp:582), then a stable sort by
// penalty (ga.cpp:583). Penalties compare as unsigned: the -1 of an invalid
// genome (tt_eval's sentinel, which the reference cannot produce) ranks last.
void tto_ga_replace(const void* p, uint8_t* pop_slot, uint8_t* pop_room, int32_t* hcv, int32_t* scv, uint8_t* feas,
                    int32_t* pen, int N, const uint8_t* cs, const uint8_t* cr, const int32_t* ch, const int32_t* csc,
                    const uint8_t* cf, const int32_t* cp, int C) {
    const Problem& P = *(const Problem*)p;
    const int E = P.E, k = N - C;
    for (int c = 0; c < C; c++) {
        memcpy(pop_slot + (size_t)(k + c) * E, cs + (size_t)c * E, E);
        memcpy(pop_room + (size_t)(k + c) * E, cr + (size_t)c * E, E);
        hcv[k + c] = ch[c]; scv[k + c] = csc[c]; feas[k + c] = cf[c]; pen[k + c] = cp[c];
    }
    std::vector<int> idx(N);
    for (int i = 0; i < N; i++) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return (uint32_t)pen[a] < (uint32_t)pen[b]; });
    std::vector<uint8_t> s2((size_t)N * E), r2((size_t)N * E), f2(N);
    std::vector<int32_t> h2(N), sc2(N), p2(N);
    for (int i = 0; i < N; i++) {
        memcpy(&s2[(size_t)i * E], pop_slot + (size_t)idx[i] * E, E);
        memcpy(&r2[(size_t)i * E], pop_room + (size_t)idx[i] * E, E);
        h2[i] = hcv[idx[i]]; sc2[i] = scv[idx[i]]; f2[i] = feas[idx[i]]; p2[i] = pen[idx[i]];
    }
    memcpy(pop_slot, s2.data(), s2.size());
    memcpy(pop_room, r2.data(), r2.size());
    for (int i = 0; i < N; i++) { hcv[i] = h2[i]; scv[i] = sc2[i]; feas[i] = f2[i]; pen[i] = p2[i]; }
}

// Single move primitives for unit tests (Move1/2/3, Solution.cpp:357-439).
void tto_move(const void* p, uint8_t* slot, uint8_t* room, int type, int a, int b, int c) {
    const Problem& P = *(const Problem*)p;
    Sol s;
    load(P, s, slot, room);
    if (type == 1) move1(P, s, a, b);
    else if (type == 2) move2(P, s, a, b);
    else move3(P, s, a, b, c);
    store(P, s, slot, room);
}

// Delta evaluators for unit tests (Solution.cpp:173-355); out[0..5] =
// eventHcv, eventAffectedHcv, affectedRoomInTimeslotHcv(slot(e)), eventScv,
// singleClassesScv.
void tto_event_terms(const void* p, const uint8_t* slot, const uint8_t* room, int e, int32_t* out) {
    const Problem& P = *(const Problem*)p;
    Sol s;
    load(P, s, slot, room);
    out[0] = event_hcv(P, s, e);
    out[1] = event_affected_hcv(P, s, e);
    out[2] = affected_room_in_timeslot_hcv(s, s.slot[e]);
    out[3] = event_scv(P, s, e);
    out[4] = single_classes_scv(P, s, e);
}

}  // extern "C"

// ttga-check: checksln-style validator of printed timetables (host only, no GPU).
//
//   ttga-check instance.tim [output.jsonl | -]
//
// For every `solution` line of a run (ga.cpp:169-197: from ttga-ga,
// python -m ttga.islands or the reference itself) that carries a timetable,
// recomputes hcv, scv and feasibility from the instance alone with the
// reference's definitions (Solution.cpp:63-160) and compares them with the
// printed totalBest / feasible. Prints one JSON report per solution line;
// exit status 0 iff every line agrees.
//
// Derived data as Problem.cpp:33-95; cost as the reference's loops: per slot
// the ascending event list (timeslot_events), per student and day the
// attended slots.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

namespace {

struct Instance {
    int E = 0, R = 0, F = 0, S = 0;
    std::vector<int> room_size, A, room_feat, event_feat;   // A: S x E (Problem.h:41)
    std::vector<int> student_number, possible;              // [E], [E x R]
    std::vector<std::vector<int>> events_of_student;        // student -> attended events
    std::vector<unsigned char> corr;                        // [E x E]
};

[[noreturn]] void die(const std::string& m) {
    std::cerr << "ttga-check: " << m << std::endl;
    std::exit(2);
}

// Problem::Problem(istream&) token order (Problem.cpp:7-74) and derived data (:33-95)
Instance read_tim(const std::string& path) {
    std::ifstream in(path);
    if (!in) die("cannot open " + path);
    Instance I;
    if (!(in >> I.E >> I.R >> I.F >> I.S)) die("truncated .tim header");
    auto rd = [&](std::vector<int>& v, long n) {
        v.resize(n);
        for (long i = 0; i < n; i++)
            if (!(in >> v[i])) die("truncated .tim body");
    };
    rd(I.room_size, I.R);
    rd(I.A, (long)I.S * I.E);
    rd(I.room_feat, (long)I.R * I.F);
    rd(I.event_feat, (long)I.E * I.F);
    I.student_number.assign(I.E, 0);
    I.events_of_student.assign(I.S, {});
    for (int s = 0; s < I.S; s++)
        for (int e = 0; e < I.E; e++)
            if (I.A[(long)s * I.E + e] == 1) { I.student_number[e]++; I.events_of_student[s].push_back(e); }
    I.corr.assign((size_t)I.E * I.E, 0);
    for (int s = 0; s < I.S; s++)
        for (int a : I.events_of_student[s])
            for (int b : I.events_of_student[s]) I.corr[(size_t)a * I.E + b] = 1;
    I.possible.assign((size_t)I.E * I.R, 0);
    for (int e = 0; e < I.E; e++)
        for (int r = 0; r < I.R; r++) {
            if (I.room_size[r] < I.student_number[e]) continue;
            int f = 0;
            for (; f < I.F; f++)
                if (I.event_feat[(long)e * I.F + f] == 1 && I.room_feat[(long)r * I.F + f] == 0) break;
            if (f == I.F) I.possible[(size_t)e * I.R + r] = 1;
        }
    return I;
}

struct Cost { int hcv = 0, scv = 0; };

Cost evaluate(const Instance& I, const std::vector<int>& slot, const std::vector<int>& room) {
    const int E = I.E;
    std::vector<std::vector<int>> lists(45);               // timeslot_events, ascending event
    for (int e = 0; e < E; e++) lists[slot[e]].push_back(e);
    Cost c;
    // computeHcv (Solution.cpp:141-160)
    for (int t = 0; t < 45; t++) {
        const std::vector<int>& L = lists[t];
        for (size_t i = 0; i < L.size(); i++)
            for (size_t j = i + 1; j < L.size(); j++) {
                if (room[L[i]] == room[L[j]]) c.hcv++;
                if (I.corr[(size_t)L[i] * E + L[j]]) c.hcv++;
            }
    }
    for (int e = 0; e < E; e++)
        if (!I.possible[(size_t)e * I.R + room[e]]) c.hcv++;
    // computeScv (Solution.cpp:86-139)
    for (int e = 0; e < E; e++)
        if (slot[e] % 9 == 8) c.scv += I.student_number[e];
    for (int s = 0; s < I.S; s++) {
        bool att[45] = {};
        for (int e : I.events_of_student[s]) att[slot[e]] = true;
        for (int d = 0; d < 5; d++) {
            int run = 0, n = 0;
            for (int k = 0; k < 9; k++) {
                if (att[9 * d + k]) {
                    n++;
                    if (++run > 2) c.scv++;
                } else {
                    run = 0;
                }
            }
            if (n == 1) c.scv++;
        }
    }
    return c;
}

// integer array after "key":[ in a compact JSON line
bool int_array(const std::string& ln, const char* key, std::vector<int>& out) {
    const std::string k = std::string("\"") + key + "\":[";
    size_t p = ln.find(k);
    if (p == std::string::npos) return false;
    p += k.size();
    out.clear();
    while (p < ln.size() && ln[p] != ']') {
        char* end = nullptr;
        out.push_back((int)std::strtol(ln.c_str() + p, &end, 10));
        p = end - ln.c_str();
        if (p < ln.size() && ln[p] == ',') p++;
    }
    return true;
}

bool int_field(const std::string& ln, const char* key, long& v) {
    const std::string k = std::string("\"") + key + "\":";
    const size_t p = ln.find(k);
    if (p == std::string::npos) return false;
    v = std::strtol(ln.c_str() + p + k.size(), nullptr, 10);
    return true;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2 || argc > 3) {
        std::cerr << "usage: ttga-check instance.tim [output.jsonl | -]" << std::endl;
        return 2;
    }
    const Instance I = read_tim(argv[1]);
    std::ifstream file;
    if (argc == 3 && std::strcmp(argv[2], "-")) {
        file.open(argv[2]);
        if (!file) die(std::string("cannot open ") + argv[2]);
    }
    std::istream& in = file.is_open() ? file : std::cin;
    std::string ln;
    int lines = 0, bad = 0;
    while (std::getline(in, ln)) {
        if (ln.rfind("{\"solution\":", 0) != 0) continue;
        lines++;
        long proc = -1, claimed = 0;
        int_field(ln, "procID", proc);
        int_field(ln, "totalBest", claimed);
        const bool claimed_feasible = ln.find("\"feasible\":true") != std::string::npos;
        std::vector<int> slot, room;
        if (!int_array(ln, "timeslots", slot) || !int_array(ln, "rooms", room)) {
            const bool ok = !claimed_feasible;             // infeasible lines carry no timetable (ga.cpp:189-196)
            bad += !ok;
            std::printf("{\"checked\":false,\"ok\":%s,\"procID\":%ld}\n", ok ? "true" : "false", proc);
            continue;
        }
        bool valid = (int)slot.size() == I.E && (int)room.size() == I.E;
        for (int e = 0; valid && e < I.E; e++) valid = slot[e] >= 0 && slot[e] < 45 && room[e] >= 0 && room[e] < I.R;
        if (!valid) {
            bad++;
            std::printf("{\"checked\":false,\"ok\":false,\"procID\":%ld,\"error\":\"malformed timetable\"}\n", proc);
            continue;
        }
        const Cost c = evaluate(I, slot, room);
        const bool feasible = c.hcv == 0;
        const long value = feasible ? c.scv : (long)c.hcv * 1000000 + c.scv;
        const bool ok = feasible == claimed_feasible && value == claimed;
        bad += !ok;
        std::printf("{\"checked\":true,\"claimed\":%ld,\"feasible\":%s,\"hcv\":%d,\"ok\":%s,\"procID\":%ld,\"scv\":%d,"
                    "\"value\":%ld}\n",
                    claimed, feasible ? "true" : "false", c.hcv, ok ? "true" : "false", proc, c.scv, value);
    }
    return lines > 0 && bad == 0 ? 0 : 1;
}

"""Round-5 evidence: the JSON records of this round's GPU runs (gpurun_out/r05_*,
scratch) copied into profiles/ (tracked). A/B timings and GA runs become one
JSON-lines file per study; profiles, PMC summaries and kernel statistics are
copied as they are."""
import json
import pathlib
import shutil

REPO = pathlib.Path(__file__).resolve().parent.parent
G = REPO / "gpurun_out"
P = REPO / "profiles"


def last_json(path: pathlib.Path):
    t = path.read_text()
    for ln in reversed([ln for ln in t.splitlines() if ln.startswith("{")]):
        try:
            return json.loads(ln)
        except json.JSONDecodeError:
            break                                  # an indented record: parse it whole
    return json.loads(t[t.index("{"):t.rindex("}") + 1])


def jsonl(name: str, files):
    out = []
    for f in files:
        if f.exists():
            d = last_json(f)
            d["_run"] = f"{f.parent.name}/{f.stem}"
            out.append(json.dumps(d))
    if out:
        (P / name).write_text("\n".join(out) + "\n")
        print(name, len(out))


def ga_rows(run: str, pattern: str):
    rows = []
    for f in sorted((G / run).glob(pattern)):
        d = last_json(f)
        rows.append({"run": f"{run}/{f.stem}", "config": d["config"], "gpu_children_per_s": d["gpu_children_per_s"],
                     "feasible_fraction_at_start": d["feasible_fraction_at_start"],
                     "feasible_fraction": d["feasible_fraction"], "gens": d["gens"],
                     **({"children_match_reference": d["children_match_reference"]} if "children_match_reference" in d else {})})
    return rows


def main():
    # the wide path's record loads: naive compiler loads, then pinned
    jsonl("r05_ab_lanes_records.jsonl", [G / "r05_a/ab_r5_syn.log", G / "r05_a/ab_r5_med.log",
                                          G / "r05_b/ab_r5b_syn.log"])
    # eval_corr's build phase without the per-event gene branch, 24-bit multiplies (not kept)
    jsonl("r05_ab_corr_build_branchfree.jsonl", [G / "r05_t/ab_cb_syn.log", G / "r05_t/ab_cb_med.log"])
    # the wide path with a falling per-wave issue priority (TT_LANES_PRIO, not kept)
    jsonl("r05_ab_lanes_prio.jsonl", [G / "r05_l/ab_lp_syn.log"])
    # tile6 and the tile5 priority schedules / grid
    jsonl("r05_ab_tile6.jsonl", [G / "r05_b/ab_r5b_med.log", G / "r05_b/ab_r5b_lg.log", G / "r05_b/ab_r5b_comp01.log",
                                 G / "r05_c/t6_ablate.log", G / "r05_d/ab_t5d_med.log", G / "r05_d/ab_t5d_lg.log",
                                 G / "r05_d/ab_t5d_comp01.log", G / "r05_d/t6_ablate.log"])
    jsonl("r05_ab_tile5_prio.jsonl", [G / f"r05_e/ab_prio_{c}.log" for c in ("med", "lg", "comp01")] +
          [G / f"r05_f/ab_prio2_{c}.log" for c in ("med", "lg", "comp01")])
    jsonl("r05_ab_tile5_grid.jsonl", [G / f"r05_i/ab_grid_{c}.log" for c in ("med", "lg")] +
          [G / f"r05_k/ab_prio3_{c}.log" for c in ("med", "lg", "comp01")] +
          [G / f"r05_j/ab_grid2_{c}.log" for c in ("med", "lg", "comp01", "med262k", "sm")])
    # local search: pair bounds on the GA (P1B builds against P1B=0 builds, same box)
    rows = []
    for run, pat in (("r05_b", "ga8k_comp*_r5b*.log"), ("r05_c", "ga8k_comp*_r5c*.log"), ("r05_d", "ga8k_comp*_r5d*.log"),
                     ("r05_f", "ga8k_comp*_r5f*.log"), ("r05_g", "ga8k_comp*_r5g*.log"), ("r05_h", "ga8k_comp*_r5*.log"),
                     ("r05_e", "ga8k_comp01_*.log")):
        rows += ga_rows(run, pat)
    (P / "r05_ab_ls_pair_bounds_ga.jsonl").write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    print("r05_ab_ls_pair_bounds_ga.jsonl", len(rows))
    # compact matcher tasks (tc1) against the round-4 task layout (tc0) and 6 waves per SIMD (w6)
    jsonl("r05_ab_ls_task_compact.jsonl", [G / f"r05_o/ab_ls_{c}.log" for c in ("comp01_8192", "med_4096", "med_65536", "lg_8192")])
    rows = ga_rows("r05_n", "ga8k_comp*_tc*.log") + ga_rows("r05_o", "ga8k_comp*.log")
    (P / "r05_ab_ga_task_compact.jsonl").write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    # the build after the compact tasks and the stream islands: bench, LS, GA (tests 234 green in the same call)
    # r05_x: the final build (the phase-2 mask policy, deferred island logging; 235 GPU tests green)
    for run in ("r05_r", "r05_x"):
        for src, dst in (("bench", "bench"), ("bench_ls", "ls200"), ("bench_ls1000", "ls1000"), ("ga8k", "ga8k"),
                         ("ga32k", "ga32k"), ("bench_syn", "bench_syn")):
            f = G / run / f"{src}.log"
            if f.exists():
                (P / f"{run}_{dst}.json").write_text(json.dumps(last_json(f), indent=1))
        for src, dst in (("prof", "bench"), ("prof_syn", "bench_syn")):
            f = G / run / src / "run_kernel_stats.csv"
            if f.exists():
                shutil.copy(f, P / f"{run}_{dst}_kernel_stats.csv")
    for src, dst in (("r05_y/ga_comps.json", "r05_y_ga_comps20.json"), ("r05_y/ga_comps_isl2.json", "r05_y_ga_comps20_islands2.json")):
        if (G / src).exists():
            shutil.copy(G / src, P / dst)
    # LS occupancy against the phase-2 student masks on the GA (r05_u/v), then the adaptive policy (r05_w)
    rows = ga_rows("r05_u", "ga8k_comp*.log") + ga_rows("r05_v", "ga8k_comp*.log")
    (P / "r05_ab_ga_ls_masks.jsonl").write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    jsonl("r05_ab_ls_wpe4.jsonl", [G / "r05_u/ab_ls_comp01_8192.log", G / "r05_u/ab_ls_med_65536.log"])
    rows = ga_rows("r05_w", "ga8k_comp*.log")
    for r in rows:
        r["ls_phase2_step_share"] = last_json(G / (r["run"] + ".log")).get("ls_phase2_step_share")
    (P / "r05_ab_ga_mask_policy.jsonl").write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    # LS issue priority rising with a wave's steps (TT_LS_PRIO 128 / 64; not kept)
    rows = ga_rows("r05_pr", "ga8k_comp*.log")
    (P / "r05_ab_ga_ls_step_prio.jsonl").write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    jsonl("r05_ab_ls_step_prio.jsonl", [G / "r05_pr/ab_ls_comp01_8192.log", G / "r05_pr/ab_ls_med_65536.log"])
    # islands multiplexed on one GPU, each on its own stream (bench_ga --islands K)
    rows = ga_rows("r05_q", "ga8k_comp*_isl*.log") + ga_rows("r05_r", "ga8k_comp*_isl*.log") + \
        ga_rows("r05_y", "ga8k_comp*_isl*.log") + ga_rows("r05_i3", "ga8k_comp*_isl*.log") + \
        ga_rows("r05_i4q", "ga8k_comp*_isl*.log")
    for r in rows:
        r["islands"] = int(r["run"].rsplit("isl", 1)[1])
        if r["run"].startswith("r05_i4q/"):
            r["env"] = "GPU_MAX_HW_QUEUES=8"     # the other runs: HIP's default, 4 hardware queues
    (P / "r05_ga8k_islands_streams.jsonl").write_text("\n".join(json.dumps(r) for r in rows) + "\n")
    if (G / "r05_p/occ_sweep.log").exists():
        shutil.copy(G / "r05_p/occ_sweep.log", P / "r05_occ_sweep.jsonl")
    jsonl("r05_ab_ls_poss16.jsonl", [G / f"r05_p/ab_ls_{c}.log" for c in ("comp01_8192", "med_65536")])
    if (G / "r05_n/occ_probe.log").exists():
        shutil.copy(G / "r05_n/occ_probe.log", P / "r05_occ_probe.jsonl")
    for src, dst in (("r05_b/ga8k_comp15_check.log", "r05_ga8k_comp15_bitexact.json"),):
        if (G / src).exists():
            (P / dst).write_text(json.dumps(last_json(G / src), indent=1))
    # section profiles and PMC of the phase-1-bound GA, before and after
    for run, tag in (("r05_a", "before"), ("r05_i", "after")):
        for c in ("comp15", "comp10"):
            f = G / run / f"lsprof_ga_{c}.log"
            if f.exists():
                (P / f"r05_lsprof_ga_{c}_{tag}.json").write_text(json.dumps(last_json(f), indent=1))
            f = G / run / f"pmc_ga_{c}.json"
            if f.exists():
                shutil.copy(f, P / f"r05_pmc_ls_ga_{c}_{tag}.json")
    for f in (G / "r05_e").glob("lsprof_comp01_*.log"):
        (P / f"r05_{f.stem}.json").write_text(json.dumps(last_json(f), indent=1))
    f = G / "r05_f/ga_trace15/run_kernel_stats.csv"
    if f.exists():
        shutil.copy(f, P / "r05_ga8k_comp15_kernel_stats.csv")


if __name__ == "__main__":
    main()

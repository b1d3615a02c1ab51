"""BASELINE configs[2] as one table: the full GA (tools/bench_ga.py's run_ga:
pop 65,536, 8,192 children per generation, maxSteps 1000, up to 96 untimed
generations or 60 % feasible, then >= 1 s timed) on every comp-size instance
comp01..comp20 in one process, each with its 512-child bit-exact check
against the reference's per-child path (oracle/_ref, ga.cpp:543-577).

    python tools/ga_comps.py OUT.json [comp01 comp05 ...]
"""
import json
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent))
import bench_ga  # noqa: E402

out_path = pathlib.Path(sys.argv[1])
names = sys.argv[2:] or [f"comp{i:02d}" for i in range(1, 21)]
rows = []
for name in names:
    a = bench_ga.parser().parse_args(["--config", name, "--pop", "65536", "--children", "8192", "--steps", "1000",
                                      "--warm-gens", "96", "--warm-feasible", "0.6", "--gens", "25",
                                      "--min-seconds", "1.0", "--cpu-sample", "512"])
    r = bench_ga.run_ga(a)
    m = r.get("children_match_reference", {})
    row = {"config": name, "E": r["E"], "R": r["R"], "S": r["S"], "gpu_children_per_s": r["gpu_children_per_s"],
           "generations_timed": r["gens"], "warm_gens": r["warm_gens"],
           "feasible_at_start": r["feasible_fraction_at_start"], "feasible_at_end": r["feasible_fraction"],
           "best_scv_feasible": r["best_scv_feasible"], "children_bit_exact": m.get("match"),
           "cpu_children_per_s": r.get("cpu_baseline", {}).get("children_per_s")}
    rows.append(row)
    print(json.dumps(row), flush=True)
    out_path.write_text(json.dumps({"rows": rows, "workload": "pop 65536, 8192 children/gen, maxSteps 1000, "
                                                             "<= 96 warm generations (or 60 % feasible), >= 1 s timed",
                                    "cpu": "reference per-child path on the box's granted cores, 512-child sample"},
                                   indent=1))

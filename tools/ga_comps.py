"""BASELINE configs[2] as one table: the full GA (tools/bench_ga.py's run_ga:
pop 65,536, 8,192 children per generation, maxSteps 1000, up to 96 untimed
generations or 60 % feasible, then >= 1 s timed) on every comp-size instance
comp01..comp20 in one process, each with its 512-child bit-exact check
against the reference's per-child path (oracle/_ref, ga.cpp:543-577).

    python tools/ga_comps.py OUT.json [--islands K] [--schedule staggered] [comp01 comp05 ...]

--islands K: K islands of 65,536 on their own streams (tools/bench_ga.py --islands),
children/s over all K; the bit-exact check covers island 0's children.
"""
import json
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent))
import bench_ga  # noqa: E402

out_path = pathlib.Path(sys.argv[1])
args = sys.argv[2:]
islands = 1
if "--islands" in args:
    i = args.index("--islands")
    islands = int(args[i + 1])
    del args[i:i + 2]
schedule = "batch"
if "--schedule" in args:
    i = args.index("--schedule")
    schedule = args[i + 1]
    del args[i:i + 2]
names = args or [f"comp{i:02d}" for i in range(1, 21)]
rows = []
for name in names:
    a = bench_ga.parser().parse_args(["--config", name, "--pop", "65536", "--children", "8192", "--steps", "1000",
                                      "--warm-gens", "96", "--warm-feasible", "0.6", "--gens", "25",
                                      "--min-seconds", "1.0", "--cpu-sample", "512", "--islands", str(islands),
                                      "--schedule", schedule])
    r = bench_ga.run_ga(a)
    m = r.get("children_match_reference", {})
    row = {"config": name, "islands": islands, "schedule": schedule, "E": r["E"], "R": r["R"], "S": r["S"], "gpu_children_per_s": r["gpu_children_per_s"],
           "generations_timed": r["gens"], "warm_gens": r["warm_gens"],
           "feasible_at_start": r["feasible_fraction_at_start"], "feasible_at_end": r["feasible_fraction"],
           "best_scv_feasible": r["best_scv_feasible"], "children_bit_exact": m.get("match"),
           "cpu_children_per_s": r.get("cpu_baseline", {}).get("children_per_s")}
    rows.append(row)
    print(json.dumps(row), flush=True)
    out_path.write_text(json.dumps({"rows": rows, "workload": f"{islands} island(s) ({schedule} schedule) of pop 65536 (one stream each when > 1), 8192 children/gen, maxSteps 1000, "
                                                             "<= 96 warm generations (or 60 % feasible), >= 1 s timed",
                                    "cpu": "reference per-child path on the box's granted cores, 512-child sample"},
                                   indent=1))

"""Where eval_tile5's LDS bank conflicts and VALU instructions come from
(profiling only): an ablation build (-DTT_EVAL_ABLATE=1, tools/ab_build.sh)
runs the headline workload once per variant under `rocprofv3 --pmc`, each
variant switching one wave-phase component off (results invalid); per
individual: LDS-array cycles, bank-conflict cycles, LDS and VALU instructions.
The difference to the full kernel is the component's share.

    python tools/t5_components.py ab_libs/libttga_abl.so [med] [65536]
    (child mode: python tools/t5_components.py --child LIB CFG P VARIANT)
"""
import json
import os
import pathlib
import sys

REPO = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "timetabling-ga-mpi-openmp_amd"))
sys.path.insert(0, str(REPO / "tools"))

# tt_eval_variant profiling bits (csrc/tt_eval.hip): 1 lane phase, 2 wave phase, 4 correlation
# words, 8 B-bitset atomics, 16 cell-counter atomics, 32 workspace zeroing
PARTS = {"full": 0, "no_lane_phase": 1, "no_wave_phase": 2, "no_corr_words": 4, "no_bitset_atomics": 8,
         "no_cell_atomics": 16, "no_ws_zeroing": 32}
COUNTERS = "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"


def child(lib, cfg, P, variant):
    import torch

    import ttga
    from ttga import native
    native._lib = native.load(pathlib.Path(lib).resolve())
    inst = ttga.config_instance(cfg)
    dp = native.DeviceProblem(inst)
    seeds = torch.from_numpy(ttga.population_seeds(12345, P)).cuda()
    slot = torch.empty((P, inst.E), dtype=torch.uint8, device="cuda")
    room = torch.empty_like(slot)
    dp.random_init(seeds, slot, room)
    out = dp.eval(slot, room, variant=8)
    for _ in range(20):
        dp.eval(slot, room, variant=8 | (variant << 4), out=out)
    torch.cuda.synchronize()


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]))
        return
    import pmc_live
    lib = sys.argv[1]
    cfg = sys.argv[2] if len(sys.argv) > 2 else "med"
    P = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
    pmc_live.PASSES = {"sq": COUNTERS}
    res = {"config": cfg, "P": P, "lib": lib, "parts": {}}
    for name, bits in PARTS.items():
        c = pmc_live.collect([__file__, "--child", lib, cfg, str(P), str(bits)], "eval_tile5_kernel")
        if c is None:
            res["parts"][name] = None
            continue
        cyc = c["GRBM_GUI_ACTIVE"] / pmc_live.XCDS
        res["parts"][name] = {"lds_cycles_per_ind": c["SQ_LDS_IDX_ACTIVE"] / P,
                              "conflict_cycles_per_ind": c["SQ_LDS_BANK_CONFLICT"] / P,
                              "lds_insts_per_ind": c["SQ_INSTS_LDS"] / P, "valu_per_ind": c["SQ_INSTS_VALU"] / P,
                              "salu_per_ind": c["SQ_INSTS_SALU"] / P, "launch_cycles": cyc}
        print(name, json.dumps(res["parts"][name]), file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

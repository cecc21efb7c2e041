#!/usr/bin/env python3
"""Fold a `tools/gpu/run.sh flops:C:E` pass (rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32
and the FP32 instruction classes) into profiles/valu_flops.json: the FP32
floating-point work each kernel of a config / engine launch actually executed,
per dispatch (warm-up quarter dropped), beside SURVEY.md 8(d)'s flop model.

    python tools/summarize_flops.py <pmc-dir> <config> <engine> <frames-per-launch> \
        <survey-model-flops-per-loc> [profiles/valu_flops.json]
"""
import datetime
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_pmc import per_kernel  # noqa: E402

COUNTERS = ("SQ_INSTS_VALU_FLOPS_FP32", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32",
            "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU", "SQ_WAVES")


def main():
    src, cfg, eng, frames, model = sys.argv[1:6]
    dst = sys.argv[6] if len(sys.argv) > 6 else "profiles/valu_flops.json"
    path = os.path.join(src, f"flops_c{cfg}_{eng}", "run_counter_collection.csv")
    per = {c: per_kernel(path, c) for c in COUNTERS}
    kernels = {}
    for k in sorted(per["SQ_INSTS_VALU_FLOPS_FP32"]):
        if k.startswith("at::") or "native" in k:
            continue  # torch's own kernels (synthetic data generation)
        e = {}
        for c in COUNTERS:
            v = per[c].get(k, [])
            e[c] = sum(v) / len(v) if v else None
        e["dispatches"] = len(per["SQ_INSTS_VALU_FLOPS_FP32"][k])
        kernels[k] = e
    # the launch's kernels: dispatched once per bench step (a kernel dispatched far
    # fewer times -- the parity report's DIRECT run -- is not part of the launch)
    top = max(v["dispatches"] for v in kernels.values())
    launch = {k: v for k, v in kernels.items() if v["dispatches"] * 2 >= top}
    # SQ_INSTS_VALU_FLOPS_FP32 adds each wave instruction's per-lane FP32 flop
    # count once (v_pk_fma_f32 4, v_fma_f32 / v_pk_add_f32 2, v_add_f32 1):
    # k_p1k_lean's 9,891 per wave match its static opcode histogram
    # (profiles/r05_c2_isa_opcode_classes.txt); x 64 lanes = the wave's flops
    fl = 64.0 * sum(v["SQ_INSTS_VALU_FLOPS_FP32"] or 0 for v in launch.values())
    out = json.load(open(dst)) if os.path.exists(dst) else {}
    out["note"] = ("per dispatch averages (kernels); SQ_INSTS_VALU_FLOPS_FP32 (gfx950 event 82, 'FLOPS per instruction "
                   "on float 32 excluding MFMA') is the FP32 work the kernels executed -- the pruned "
                   "inverse, the front end and the grid as built -- beside SURVEY.md 8(d)'s model "
                   "(forward + PHAT + FULL inverse FFTs); bench.py's valu_roofline.executed prices it")
    out[f"c{cfg}_{eng}"] = {
        "date": datetime.date.today().isoformat(),
        "frames_per_launch": int(frames),
        "executed_fp32_flops_per_launch": fl,
        "executed_fp32_flops_per_loc": fl / int(frames),
        "survey_model_flops_per_loc": float(model),
        "executed_over_model": fl / int(frames) / float(model),
        "launch_kernels": sorted(launch),
        "counter_unit": "per-lane flops per wave instruction (x 64 lanes for the totals above; exec-masked "
                        "lanes of an instruction count as executed)",
        "kernels": kernels,
    }
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out[f"c{cfg}_{eng}"], indent=1))


if __name__ == "__main__":
    main()

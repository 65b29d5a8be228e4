"""HBM traffic of a training step's kernels from two rocprofv3 PMC passes
(FETCH_SIZE, WRITE_SIZE; one counter family per pass, MI355X_MICROARCH.md
§HBM), against the algorithmic bytes of the C-ABI calls that launch them
(tools/train_roofline.py's committed step JSON).

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d <f> -o run -- python3 tools/train_steps.py --kind mnv3 --steps 2
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d <w> -o run -- python3 tools/train_steps.py --kind mnv3 --steps 2
  python3 tools/pmc_train.py <f> <w> --steps 3 --roof profiles/r04/c4_step_roofline.json --out x.json

FETCH_SIZE / WRITE_SIZE are KiB; gfx950 correction: HBM bytes = 2 * FETCH_SIZE
+ WRITE_SIZE (FETCH_SIZE counts half of a 16-B-per-lane streaming read).
Counts are summed over every dispatch of the run and divided by --steps (the
train_steps run's warm-up + timed steps).  Families map kernel names to the
C-ABI call whose algorithmic bytes they implement; a ratio well above 1
means re-reads (L2 misses on data the kernel should touch once).
"""
import argparse
import collections
import csv
import glob
import json

# C-ABI call -> kernel-name substrings it launches (the BN backward kernels
# serve two calls: their algorithmic bytes are the two calls' sum)
FAMILIES = {
    "dw_dgrad_bn (jabd_dw_dgrad_bn_bwd_f32)": (["jabd_dw_dgrad_bn_bwd_f32"], ["dw_dgrad_bn_kernel"]),
    "bn_act_bwd (jabd_bn_act_bwd_ex_f32 + jabd_bn_act_bwd_f32 + _rows)":
        (["jabd_bn_act_bwd_ex_f32", "jabd_bn_act_bwd_f32", "jabd_bn_act_bwd_rows_f32"],
         ["bn_bwd_part_kernel", "bn_bwd_apply_kernel", "bn_bwd_final_kernel", "bn_rows_sum_kernel"]),
    "conv_wgrad (jabd_conv_wgrad_f32 + _eca)": (["jabd_conv_wgrad_f32", "jabd_conv_wgrad_eca_f32"],
                                               ["conv_wgrad32_kernel", "conv_wgrad_v_kernel",
                                                "wgrad_reduce2_kernel", "wgrad_img_reduce",
                                                "wgrad_eca_reduce"]),
    # the GEMM kernels serve the plain conv call and its statistics / BatchNorm-backward forms
    "conv2d_nhwc (jabd_conv2d_nhwc_f32 + _bn_stats + _bn_bwd_sums)":
        (["jabd_conv2d_nhwc_f32", "jabd_conv1x1_bn_stats_f32", "jabd_conv_bn_stats_f32",
          "jabd_conv_bn_bwd_sums_f32", "jabd_conv_bn_bwd_sums_res_f32"],
         ["conv1x1_m32_kernel", "conv1x1_m32s_kernel", "conv1x1_kernel", "conv1x1_stream_kernel", "conv3x3_tile_kernel",
          "conv_gemm_kernel", "stem7_fwd_kernel", "m32_ksplit_reduce", "bn_rows_chunk_kernel"]),
    "nlm_bwd_attn (jabd_nlm_bwd_attn_f32)": (["jabd_nlm_bwd_attn_f32"], ["nlm_bwd_attn"]),
    "bn_act_fwd (jabd_bn_act_fwd_f32 + _sum)": (["jabd_bn_act_fwd_f32", "jabd_bn_act_fwd_sum_f32"],
                                               ["bn_act_fwd_kernel", "bn_act_fwd_sum_kernel"]),
    "bn_stats (jabd_bn_stats_f32)": (["jabd_bn_stats_f32"], ["bn_stats_part_kernel"]),
    "dw_wgrad (jabd_dw_wgrad_f32 + _bnin)": (["jabd_dw_wgrad_f32", "jabd_dw_wgrad_bnin_f32"],
                                            ["dw_wgrad_strip_kernel", "dw_wgrad_rows_kernel"]),
    "dwconv_stats (jabd_dwconv_stats_f32 + _bnin + jabd_dwconv_nhwc_f32)":
        (["jabd_dwconv_stats_f32", "jabd_dwconv_bnin_stats_f32", "jabd_dwconv_nhwc_f32"],
         ["dw_rows_kernel", "dw_kernel<", "bn_stats_final_kernel"]),
}


def counters(d, name):
    out = collections.defaultdict(float)
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"].startswith(name):
                out[r.get("Kernel_Name", "")] += float(r["Counter_Value"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--steps", type=float, required=True)
    ap.add_argument("--roof", required=True)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    fe, wr = counters(a.fetch, "FETCH_SIZE"), counters(a.write, "WRITE_SIZE")
    roof = json.load(open(a.roof))
    by_call = roof["by_call"]
    rows = {}
    for fam, (calls, kerns) in FAMILIES.items():
        f = sum(v for k, v in fe.items() if any(s in k for s in kerns)) / a.steps
        w = sum(v for k, v in wr.items() if any(s in k for s in kerns)) / a.steps
        pmc_gb = (2.0 * f + w) * 1024 / 1e9
        alg_gb = sum(by_call.get(c, {}).get("mbytes", 0.0) for c in calls) / 1e3
        us = sum(by_call.get(c, {}).get("us", 0.0) for c in calls)
        rows[fam] = {"pmc_gb_per_step": pmc_gb, "fetch_gb": 2.0 * f * 1024 / 1e9,
                     "write_gb": w * 1024 / 1e9, "alg_gb_per_step": alg_gb,
                     "pmc_over_alg": pmc_gb / alg_gb if alg_gb else None,
                     "call_ms_per_step": us / 1e3,
                     "pmc_tbs": pmc_gb / (us * 1e-6) / 1e3 if us else None}
    tot_f = sum(fe.values()) / a.steps
    tot_w = sum(wr.values()) / a.steps
    res = {"workload": roof["workload"], "steps_divisor": a.steps,
           "correction": "HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (KiB), MI355X_MICROARCH.md",
           "step_total_pmc_gb": (2 * tot_f + tot_w) * 1024 / 1e9, "families": rows}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as fo:
            json.dump(res, fo, indent=1)


if __name__ == "__main__":
    main()

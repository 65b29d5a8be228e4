"""Conv-stack (conv_gemm / conv1x1 / fused expand_dw) HBM traffic per step from two rocprofv3 PMC passes.

Usage (on the GPU box, one counter per pass as MI355X_MICROARCH.md
§rocprofv3 PMC slots requires — FETCH_SIZE and WRITE_SIZE do not fit one pass):

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- \
      python3 bench.py --steps 3 --pmc-forward-only
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- \
      python3 bench.py --steps 3 --pmc-forward-only
  python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write 3 out.json

FETCH_SIZE / WRITE_SIZE are kilobytes.  gfx950 correction (MI355X_MICROARCH.md
§HBM): FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming read, so
HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE.
"""
import csv
import glob
import json
import sys

KERNELS = ("conv_gemm_kernel", "conv1x1_kernel", "conv1x1_m32_kernel", "conv1x1_stream_kernel", "conv3x3_tile_kernel", "expdw_kernel", "expdw1_kernel")  # the conv stack


def _sum(d, counter):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    tot, n = 0.0, 0
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == counter and any(k in r.get("Kernel_Name", "") for k in KERNELS):
                tot += float(r["Counter_Value"])
                n += 1
    return tot, n


def main():
    fdir, wdir, steps, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    fetch_kb, nf = _sum(fdir, "FETCH_SIZE")
    write_kb, nw = _sum(wdir, "WRITE_SIZE")
    res = {
        "conv_hbm_bytes_per_step": (2 * fetch_kb + write_kb) * 1024 / steps,
        "fetch_size_kb_per_step": fetch_kb / steps,
        "write_size_kb_per_step": write_kb / steps,
        "dispatches_per_step": nf / steps,
        "correction": "2*FETCH_SIZE (gfx950 half-count of 16B/lane reads) + WRITE_SIZE",
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, "
                  f"python3 bench.py --steps {steps} --pmc-forward-only",
    }
    assert nf == nw, (nf, nw)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

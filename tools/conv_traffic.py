"""Per-shape HBM traffic and time of the implicit-GEMM 3x3 conv at the denoise step's shapes (SDXL, 16 frames x
512^2, CFG batch 2 -> 32 images), against the algorithmic bytes (input + weights + output, each once).

  python tools/conv_traffic.py run                 # launches every shape REPS times, prints timings + order file
  rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/cpmc_f -o c -- python tools/conv_traffic.py run
  rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/cpmc_w -o c -- python tools/conv_traffic.py run
  python tools/conv_traffic.py parse gpurun_out/cpmc_f gpurun_out/cpmc_w

Counters are converted as tools/pmc_traffic.py does (fetch = 2 x 1024 x FETCH_SIZE on gfx950, write = 1024 x
WRITE_SIZE; memory-side requests, i.e. L2 misses including Infinity-Cache hits: an upper bound on HBM bytes).
Conv dispatches are matched to shapes by dispatch order (each shape runs REPS times, one after the other).
"""
import csv
import glob
import json
import os
import sys

REPS = 3
# name, nimg, H, W (input), C1, C2, Cout, mode ("" | "up" | "s2")
SHAPES = [
    ("64sq_320_320", 32, 64, 64, 320, 0, 320, ""),
    ("64sq_cat_320+320", 32, 64, 64, 320, 320, 320, ""),
    ("64sq_up_640", 32, 32, 32, 640, 0, 640, "up"),
    ("32sq_640_640", 32, 32, 32, 640, 0, 640, ""),
    ("32sq_cat_640+640", 32, 32, 32, 640, 640, 640, ""),
    ("32sq_down_320", 32, 64, 64, 320, 0, 320, "s2"),
    ("16sq_1280_1280", 32, 16, 16, 1280, 0, 1280, ""),
    ("16sq_cat_1280+1280", 32, 16, 16, 1280, 1280, 1280, ""),
]


def alg_bytes(nimg, H, W, C1, C2, Cout, mode):
    OH, OW = (2 * H, 2 * W) if mode == "up" else ((H + 1) // 2, (W + 1) // 2) if mode == "s2" else (H, W)
    M = nimg * OH * OW
    return M, 2 * (nimg * H * W * (C1 + C2) + Cout * 9 * (C1 + C2) + M * Cout)


def run():
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from video_style_transfer_amd import kernels as K
    dev = torch.device("cuda")
    BF = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    for name, nimg, H, W, C1, C2, Cout, mode in SHAPES:
        x1 = torch.randn(nimg * H * W, C1, device=dev, generator=g).to(BF)
        x2 = torch.randn(nimg * H * W, C2, device=dev, generator=g).to(BF) if C2 else None
        w = (torch.randn(Cout, 9 * (C1 + C2), device=dev, generator=g) * (9 * (C1 + C2)) ** -0.5).to(BF)
        b = torch.zeros(Cout, device=dev)
        M, ab = alg_bytes(nimg, H, W, C1, C2, Cout, mode)

        def fn():
            return K.conv3x3(x1, nimg, H, W, w, b, x2=x2, stride=2 if mode == "s2" else 1, upsample=mode == "up")
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(REPS - 1):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / (REPS - 1) * 1e3
        fl = 2.0 * M * Cout * 9 * (C1 + C2)
        print(json.dumps({"shape": name, "M": M, "N": Cout, "K": 9 * (C1 + C2), "us": round(us, 1),
                          "tflops": round(fl / us / 1e6, 1), "alg_bytes": ab,
                          "kernel": K.gemm_kernel_name(M, Cout, 9 * (C1 + C2), 2)}), flush=True)
        del x1, x2, w


def read(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") == counter and "gemm" in r["Kernel_Name"]:
                    rows.append((int(r.get("Dispatch_Id") or r.get("Correlation_Id")), float(r["Counter_Value"])))
    agg = {}
    for d_id, v in rows:
        agg[d_id] = agg.get(d_id, 0.0) + v
    return [agg[k] for k in sorted(agg)]


def parse(dfetch, dwrite):
    f, w = read(dfetch, "FETCH_SIZE"), read(dwrite, "WRITE_SIZE")
    assert len(f) == len(w) == REPS * len(SHAPES), (len(f), len(w))
    out = {}
    for i, (name, nimg, H, W, C1, C2, Cout, mode) in enumerate(SHAPES):
        fb = sum(f[i * REPS:(i + 1) * REPS]) / REPS * 2 * 1024
        wb = sum(w[i * REPS:(i + 1) * REPS]) / REPS * 1024
        _, ab = alg_bytes(nimg, H, W, C1, C2, Cout, mode)
        out[name] = {"fetch_bytes": round(fb), "write_bytes": round(wb), "alg_bytes": ab,
                     "ratio": round((fb + wb) / ab, 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(sys.argv[2], sys.argv[3])

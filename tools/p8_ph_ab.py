"""A/B of the 8-phase GEMM k-loop schedules (VST_P8_PH = 3: three barrier intervals per k-tile; 2: two) on the
denoise step's GEMM shapes, in isolation: each schedule runs in its own child process (the choice is read once per
process), alternated `passes` times; the children also hash their outputs, which must be equal (same k order).
python tools/p8_ph_ab.py [passes] [variant ...]  -> one JSON line per shape with us per launch and TF/s per variant.
A variant is the schedule, optionally '+320' for the 128x320 tile policy (VST_P8_320=1) and '+persist' for the persistent
grid (VST_P8_PERSIST=1), '+bn320' / '+bn192' to force the tile width (VST_P8_BN), '+lp' for the persistent LoRA kernels (VST_P8_LORA_PERSIST=1): e.g. 3 2 3+320 2+320 2+persist."""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SHAPES = [  # name, kind, M, N, K (16x512^2 CFG pair: 16^2 level M = 8192, 32^2 32768, 64^2 131072)
    ("geglu1280", "geglu", 8192, 10240, 1280), ("geglu640", "geglu", 32768, 5120, 640),
    ("geglu320", "geglu", 131072, 2560, 320),
    ("ff2_1280", "plain", 8192, 1280, 5120), ("ff2_640", "plain", 32768, 640, 2560), ("proj320", "plain", 131072, 320, 320),
    ("out1280_lora", "lora1", 8192, 1280, 1280), ("qkv1280_lora", "lora3", 8192, 3840, 1280),
    ("out640_lora", "lora1", 32768, 640, 640), ("qkv640_lora", "lora3", 32768, 1920, 640),
    ("qkv960_320", "plain", 131072, 960, 320), ("ff2_320", "plain", 131072, 320, 1280),
    ("xattn1280_lora", "xattn", 8192, 1280, 1280), ("xattn640_lora", "xattn", 32768, 640, 640),
]
if os.environ.get("VST_AB_SHAPES"):  # comma-separated subset of the names above
    _keep = set(os.environ["VST_AB_SHAPES"].split(","))
    SHAPES = [s for s in SHAPES if s[0] in _keep]


def child(passes_inner=2):
    import torch
    sys.path.insert(0, ROOT)
    from video_style_transfer_amd import kernels as K
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    out = []
    for name, kind, M, N, Kd in SHAPES:
        x = torch.randn(M, Kd, device=dev, generator=g).to(torch.bfloat16)
        r = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
        b = torch.randn(N, device=dev, generator=g) * 0.1
        if kind == "xattn":  # attn2: to_q + UnZipLoRA (r 8: 16 u columns) + the 77-key text attention epilogue
            P = 32
            w = (torch.randn(N, Kd + P, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
            a = torch.zeros(P, Kd, device=dev)
            a[:16] = torch.randn(16, Kd, device=dev, generator=g) * Kd ** -0.5
            a = a.to(torch.bfloat16)
            kt = torch.randn(32 * 77, N, device=dev, generator=g).to(torch.bfloat16)
            vt = torch.randn(32 * 77, N, device=dev, generator=g).to(torch.bfloat16)
            nq = M // 32
            fn = (lambda: K.linear_cross_attention(x, w, a, N, 16, b, kt, vt, Nq=nq, Nk=77, kv_div=1, scale=0.125))
            fl = 2.0 * M * N * (Kd + 16) + 2.0 * M * Kd * 16 + 4.0 * M * N * 77
        elif kind.startswith("lora"):
            nproj = int(kind[-1])
            P = 32 if nproj == 1 else 64
            w = (torch.randn(N, Kd + P, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
            a = torch.zeros(P, Kd, device=dev)
            a[:16 * nproj] = torch.randn(16 * nproj, Kd, device=dev, generator=g) * Kd ** -0.5
            a = a.to(torch.bfloat16)
            fn = (lambda: K.linear_lora(x, w, a, N // nproj, 16, b, residual=r if nproj == 1 else None))
            fl = 2.0 * M * N * (Kd + 16) + 2.0 * M * Kd * 16 * nproj
        else:
            w = (torch.randn(N, Kd, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
            geglu = kind == "geglu"
            fn = (lambda: K.linear(x, w, b, geglu=geglu, residual=None if geglu else r))
            fl = 2.0 * M * N * Kd
        try:
            y = fn()
        except K._lib.VstError:  # (the 32x32 q/k/v straddles 256-wide tiles: in-GEMM LoRA only on 128x320 tiles)
            out.append({"ph": os.environ.get("VST_P8_PH", "3"), "shape": name, "us": 1e9, "tflops": 0.0, "md5": "-",
                        "kernel": "unsupported", "lora_tile": 0})
            continue
        torch.cuda.synchronize()
        h = hashlib.md5(y.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:12]
        best = 1e9
        for _ in range(passes_inner):
            for _ in range(3):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(20):
                fn()
            e.record()
            torch.cuda.synchronize()
            best = min(best, s.elapsed_time(e) * 1e3 / 20)
        out.append({"ph": os.environ.get("VST_P8_PH", "3"), "shape": name, "M": M, "N": N, "K": Kd,
                    "lora_tile": K.gemm_lora_tile(M, N, Kd, 32 if kind == "lora1" else 64, N // int(kind[-1]), 16)
                    if kind.startswith("lora") else None,
                    "kernel": "xattn" if kind == "xattn" else None if kind.startswith("lora") else
                    K.gemm_kernel_name(M, N, Kd, 1 if kind == "geglu" else 0),
                    "us": round(best, 2), "tflops": round(fl / best / 1e6, 1), "md5": h})
    for o in out:
        print(json.dumps(o), flush=True)


def main():
    if os.environ.get("VST_PH_CHILD"):
        return child()
    passes = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    phs = sys.argv[2:] or ["3", "2"]
    res = {}
    for _ in range(passes):
        for ph in phs:
            env = dict(os.environ, VST_P8_PH=ph.split("+")[0], VST_PH_CHILD="1", VST_P8_320="1" if "+320" in ph else "0",
                       VST_P8_PERSIST="1" if "+persist" in ph else "0",
                       VST_P8_BN="320" if "+bn320" in ph else "192" if "+bn192" in ph else "0",
                       VST_P8_LORA_PERSIST="1" if "+lp" in ph else "0",
                       )
            r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True, text=True,
                               timeout=300)
            if r.returncode:
                print(r.stderr[-3000:], file=sys.stderr)
                raise SystemExit(r.returncode)
            print(f"[ab] variant {ph} done", flush=True)
            for line in r.stdout.splitlines():
                d = json.loads(line)
                key = (d["shape"], ph)
                if key not in res or d["us"] < res[key]["us"]:
                    res[key] = d
    for name, *_ in SHAPES:
        row = {ph: res[(name, ph)] for ph in phs}
        md5s = {d["md5"] for d in row.values() if d["md5"] != "-"}
        print(json.dumps({"shape": name, **{f"us_ph{ph}": d["us"] for ph, d in row.items()},
                          **{f"tf_ph{ph}": d["tflops"] for ph, d in row.items()},
                          **{f"kernel_{ph}": d["kernel"] or d["lora_tile"] for ph, d in row.items()},
                          "bitwise_equal": len(md5s) == 1}), flush=True)


if __name__ == "__main__":
    main()

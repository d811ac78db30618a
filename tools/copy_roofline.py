"""What a read+write stream of the step's HBM-bound sizes reaches on this box: device-to-device copies (torch's copy
kernel) of the LayerNorm / GroupNorm operand sizes (8192 / 32768 / 131072 rows of 1280 / 640
/ 320 bf16 = 21 / 42 / 84 MB read + as much written), back to back, timed with events; the TB/s counts read + written
bytes.  The ceiling the verdict's "HBM-bound kernels >= 5 TB/s" is measured against.
python tools/copy_roofline.py"""
import json

import torch


def main():
    dev = torch.device("cuda")
    out = []
    for rows, C in ((8192, 1280), (32768, 640), (131072, 320), (32768, 1280), (131072, 1280)):
        a = torch.randn(rows, C, device=dev).to(torch.bfloat16)
        b = torch.empty_like(a)
        nbytes = 2 * a.numel() * a.element_size()
        res = {"rows": rows, "C": C, "MB_moved": round(nbytes / 1e6, 1)}
        for name, fn in (("torch_copy", lambda: b.copy_(a)),):
            for _ in range(5):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(50):
                fn()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 1e3 / 50
            res[name + "_us"] = round(us, 2)
            res[name + "_TBs"] = round(nbytes / us / 1e6, 2)
        out.append(res)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

"""HBM traffic per launch from rocprofv3 PMC counters, per kernel (as bench.py names kernels).

Two passes (FETCH_SIZE needs 3 TCC slots and WRITE_SIZE 2, so they cannot share a pass), each run as
  rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o pmc -- python bench.py ...
  rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o pmc -- python bench.py ...
then  python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_so.md5 \
          > profiles/pmc_traffic_rN.json
(pmc_so.md5 = md5sum of the libvst_hip.so the passes ran: bench.py uses the file only for that library.)

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of wide (16 B/lane) coalesced streaming reads — every read on this path is a 16-B
buffer load or LDS-DMA — so fetched bytes = 2 x 1024 x FETCH_SIZE; WRITE_SIZE is exact for 16-B stores.
Both count Infinity-Cache hits too (memory-side request counters), so this is L2-miss traffic: an upper
bound on HBM bytes.
"""
import csv
import glob
import json
import os
import re
import sys


def bench_symbol(name: str) -> str:
    """rocprof kernel name -> the symbol bench.py / vst_gemm_kernel_name report."""
    m = re.search(r"gemm_ring_kernel<vst::RingCfg<(\d+), (\d+), \d+, \d+, \d+>, (\d), (\d)>", name)
    if m:
        bm, bn, amode, epi = m.groups()
        tag = {("0", "0"): "", ("0", "1"): ",geglu", ("1", "0"): ",conv", ("0", "2"): ",splitk",
               ("1", "2"): ",splitk"}.get((amode, epi), f",a{amode}e{epi}")
        return f"gemm_ring<{bm}x{bn}{tag}>"
    # gemm_p8_kernel<EPI, BN, LORA, PH, BM, CONV, PERSIST>
    m = re.search(r"gemm_p8_kernel<(\d), (\d+), (true|false), \d, (\d+)(?:, (true|false))?(?:, (true|false))?>", name)
    if m:
        epi, bn, lora, bm, conv, persist = m.groups()
        tags = ((",lora" if lora == "true" else "") + (",conv" if conv == "true" else "") +
                (",geglu" if epi == "1" else "") + (",xattn" if epi == "4" else "") + (",tattn" if epi == "5" else "") +
                (",persist" if persist == "true" else ""))
        return f"gemm_p8<{bm}x{bn}{tags}>"
    if "layernorm_lora_kernel" in name:
        return "layernorm_lora"
    for k, v in (("gemm_skinny", "gemm_skinny"), ("spatial_attn_kernel", "spatial_attn_kernel"),
                 ("layernorm_g_kernel", "layernorm_kernel"),
                 ("temporal_attn_kernel", "temporal_attn_kernel"), ("layernorm_kernel", "layernorm_kernel"),
                 ("gn_", "gn_stats/gn_finalize/gn_apply"), ("gemm_kernel<2", "gemm_kernel<conv_in>"),
                 ("gemm_rows_kernel", "gemm_rows")):
        if k in name:
            return v
    return name.split("(")[0][:80]


def read_counter(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = {}
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") != counter:
                    continue
                key = bench_symbol(r["Kernel_Name"])
                disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
                e = per.setdefault(key, {})
                e[disp] = e.get(disp, 0.0) + float(r["Counter_Value"])
    return per


def main():
    fetch = read_counter(sys.argv[1], "FETCH_SIZE")
    write = read_counter(sys.argv[2], "WRITE_SIZE")
    lib_md5 = open(sys.argv[3]).read().split()[0] if len(sys.argv) > 3 else None
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import src_hash
    out = {"lib_md5": lib_md5, "src_hash": src_hash(), "note": "bytes per launch; fetch = 2 x 1024 x FETCH_SIZE (gfx950 wide-read correction), "
                   "write = 1024 x WRITE_SIZE; memory-side requests (L2 misses incl. Infinity-Cache hits)",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, {}), write.get(k, {})
        if not f or not w:
            continue
        fb = 2 * 1024 * sum(f.values()) / len(f)
        wb = 1024 * sum(w.values()) / len(w)
        out["kernels"][k] = {"launches": len(f), "fetch_bytes": round(fb), "write_bytes": round(wb),
                             "traffic_bytes": round(fb + wb)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

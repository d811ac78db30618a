"""A/B of two builds of libvst_hip.so on the step's GEMM shapes (tools/p8_ph_ab.py's child: us per launch, output
md5): each build runs in its own child process (VST_LIB_AB), alternated `passes` times, best time kept.
python tools/lib_ab.py passes name=path [name=path ...]   (path "-" = the in-tree library)
VST_AB_SHAPES=a,b restricts the shapes.  One JSON line per shape: us and TF/s per build, and whether every build's
output is bit-identical."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    passes = int(sys.argv[1])
    libs = [a.split("=", 1) for a in sys.argv[2:]]
    res = {}
    order = []
    for _ in range(passes):
        for name, path in libs:
            env = dict(os.environ, VST_PH_CHILD="1", VST_P8_PH="2")
            env.pop("VST_LIB_AB", None)
            if path != "-":
                env["VST_LIB_AB"] = path
            r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "p8_ph_ab.py")], env=env,
                               capture_output=True, text=True, timeout=300)
            if r.returncode:
                print(r.stderr[-3000:], file=sys.stderr)
                raise SystemExit(r.returncode)
            print(f"[ab] {name} done", flush=True)
            for line in r.stdout.splitlines():
                if not line.startswith("{"):
                    continue
                d = json.loads(line)
                if d["shape"] not in order:
                    order.append(d["shape"])
                key = (d["shape"], name)
                if key not in res or d["us"] < res[key]["us"]:
                    res[key] = d
    for shape in order:
        row = {name: res[(shape, name)] for name, _ in libs}
        md5s = {d["md5"] for d in row.values()}
        print(json.dumps({"shape": shape, **{f"us_{n}": d["us"] for n, d in row.items()},
                          **{f"tf_{n}": d["tflops"] for n, d in row.items()}, "bitwise_equal": len(md5s) == 1}),
              flush=True)


if __name__ == "__main__":
    main()

"""Load time and peak host RSS of bert_load_from_file for 1 vs N replicas
(repack once, upload N times).

Each point runs in a fresh child process (BERT_DEVICES = the ordinal repeated N
times, so N replicas share one GPU): the child loads the model, reports the wall
time of the call and its peak RSS (ru_maxrss) before and after, runs one forward,
and exits.  `--libs name:path,...` compares builds (e.g. the previous round's
library, where every replica thread repacked the whole model on its own).

    python scripts/load_profile.py --arch bge-large-en-v1.5 --ftype q4_1 --replicas 1,8 \
        --libs new:build/libbert.so,r05:build_ab/r05/libbert.so --out gpurun_out/load.jsonl
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))

CHILD = r"""
import ctypes, json, os, resource, sys, time
sys.path.insert(0, sys.argv[1])
import numpy as np
import bertpy
L = bertpy.load_lib(sys.argv[3])
rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
t0 = time.perf_counter()
ctx = L.bert_load_from_file(sys.argv[2].encode())
t1 = time.perf_counter()
rss1 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
assert ctx, "load failed"
n = L.bertx_num_devices(ctx)
m = bertpy.BertModel.__new__(bertpy.BertModel)
m.lib, m.ctx = L, ctx
m.n_embd, m.n_max_tokens = L.bert_n_embd(ctx), L.bert_n_max_tokens(ctx)
e = m.forward_batch([np.arange(1000, 1000 + 128, dtype=np.int32)] * (4 * n))
print(json.dumps({"replicas": n, "load_s": t1 - t0, "rss_before_mib": rss0 / 1024, "rss_peak_mib": rss1 / 1024,
                  "finite": bool(np.isfinite(e).all())}), flush=True)
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="bge-large-en-v1.5")
    ap.add_argument("--ftype", default="q4_1")
    ap.add_argument("--replicas", default="1,8")
    ap.add_argument("--libs", default="new:" + os.path.join(ROOT, "build", "libbert.so"))
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="loadprof_")
    path = os.path.join(tmp, f"{a.arch}-{a.ftype}.bin")
    # the model is written by a child too: this process stays small, so the load
    # children (whose peak RSS starts from the parent's at fork) measure the load
    subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, sys.argv[1]); import bertpy; "
                    "bertpy.synthetic_model(sys.argv[2], sys.argv[3], sys.argv[4], seed=1234)",
                    os.path.join(ROOT, "embeddings.cpp_amd"), path, a.arch, a.ftype], check=True)
    size = os.path.getsize(path)
    rows = []
    for rep in range(a.repeat):
        for spec in a.libs.split(","):
            name, lib = spec.split(":", 1)
            for n in (int(x) for x in a.replicas.split(",")):
                env = dict(os.environ, BERT_DEVICES=",".join(["0"] * n))
                p = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "embeddings.cpp_amd"), path, lib],
                                   capture_output=True, text=True, env=env, timeout=600)
                if p.returncode != 0:
                    print(p.stdout[-2000:], p.stderr[-2000:], file=sys.stderr)
                    raise SystemExit(f"{name} x{n}: child failed ({p.returncode})")
                r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
                r.update(lib=name, arch=a.arch, ftype=a.ftype, file_mib=size / 2**20, repeat=rep)
                print(json.dumps(r), flush=True)
                rows.append(r)
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    os.remove(path)


if __name__ == "__main__":
    main()

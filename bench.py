#!/usr/bin/env python3
"""Benchmark of the MI355X BERT/BGE embedding forward (BASELINE.json metric).

One step = one forward of the workload's batch (bge-base-en-v1.5 architecture,
q4_0 weights, 64 sentences x 512 tokens per GPU) through libbert.so's
device-resident entry point (bertx_forward_device), with token ids already in HBM.
Multi-GPU: one process per GPU (torchrun); every rank runs its own 64-sentence
shard ("weak" scaling, no data-path collective -- the path is embarrassingly
parallel); the timed region is bracketed by barriers and the max over ranks is
reported.  Weights are synthetic (random init of the architecture, seeded) --
there are no checkpoints offline.

Prints ONE JSON line on rank 0.
"""
import argparse
import collections
import csv
import ctypes
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "embeddings.cpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

MFMA_F16_PEAK_TFLOPS = 2500.0    # MI355X dense f16/bf16 MFMA (MI355X_MICROARCH.md, chip table)
HBM_PEAK_GBPS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--arch", default="bge-base-en-v1.5")
    p.add_argument("--ftype", default="q4_0")
    p.add_argument("--batch", type=int, default=64, help="sentences per GPU")
    p.add_argument("--seq", type=int, default=512)
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--model-dir", default=os.environ.get("EMB_MODEL_DIR", "/tmp/emb_models"))
    p.add_argument("--cpu-baseline-sentences", type=int, default=24)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-profile", action="store_true", help="disable live per-kernel event timing")
    p.add_argument("--no-probes", action="store_true", help="skip the north-star probes (C2 f16, B=1 L=32 q4_0)")
    p.add_argument("--no-library", action="store_true", help="skip the host-buffer library-path measurement")
    p.add_argument("--no-pmc", action="store_true",
                   help="skip this run's rocprofv3 PMC passes (HBM bytes per kernel launch, build/bin/bert_probe)")
    p.add_argument("--inproc", action="store_true",
                   help="one process drives --gpus GPUs through bert_forward_batch (the library's own sharding, "
                        "BERT_DEVICES=0..N-1) on --inproc-batch sentences of the --inproc-arch/--inproc-ftype model "
                        "(default SURVEY C4: bge-large-en-v1.5 q4_1, L 512, 256 sentences)")
    p.add_argument("--inproc-arch", default="bge-large-en-v1.5")
    p.add_argument("--inproc-ftype", default="q4_1")
    p.add_argument("--inproc-batch", type=int, default=256)
    p.add_argument("--no-encode", action="store_true", help="skip the text-in bert_encode_batch leg")
    p.add_argument("--dry-step", action="store_true",
                   help="CPU stub in place of the forward (no GPU, gloo): tests the launch / timing / reporting "
                        "skeleton, never a measurement")
    return p.parse_args()


def launch_ranks(a):
    """`python bench.py --gpus N` (N > 1) without a torchrun environment: start the N
    rank processes here -- torch.distributed.run as a CHILD process, before this
    process has imported torch or touched a GPU (never a re-exec of a process that
    has initialised the GPU) -- and exit with its status.  Rank 0 prints the JSON
    line to the inherited stdout."""
    # --standalone: the launcher binds its own free rendezvous port (no window between
    # choosing a port here and binding it there), on 127.0.0.1
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           f"--nproc-per-node={a.gpus}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def algorithmic_bytes(hp, ftype, B, L):
    """Compulsory HBM bytes of one batch: weights at stored width,
    f32 biases/LN, gathered embedding rows, ids in, embeddings out."""
    bpw = {"f32": 4.0, "f16": 2.0, "q4_0": 0.5625, "q4_1": 0.625, "q8_0": 1.0625}[ftype]
    d, f, nl = hp["n_embd"], hp["n_intermediate"], hp["n_layer"]
    w = nl * (4 * d * d + 2 * d * f) * bpw
    small = nl * (9 * d + f) * 4 + 4 * d * 4
    emb_rows = B * L * d * bpw + L * d * bpw + 2 * d * bpw   # word row per token; position / type tables once
    return w + small + emb_rows + 4 * B * L + 4 * B * d


def timed_steps(step, steps, sync, dist=None, reduce_device="cpu", per_rank=None):
    """The contract's timed region: barrier + sync, `steps` steps, sync + barrier;
    returns the MAX over ranks of the elapsed seconds (every rank gets it).  With a
    list `per_rank`, it also receives every rank's own elapsed seconds (all_gather)."""
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        if per_rank is not None:
            mine = torch.tensor([elapsed], dtype=torch.float64, device=reduce_device)
            allv = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
            dist.all_gather(allv, mine)
            per_rank.extend(float(v.item()) for v in allv)
        tt = torch.tensor([elapsed], dtype=torch.float64, device=reduce_device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    elif per_rank is not None:
        per_rank.append(elapsed)
    return elapsed


class DeviceForward:
    """One model's device-resident forward (bertx_forward_device) on HBM-resident
    ids, captured into a HIP graph by the library on its second use."""

    def __init__(self, lib, bertpy, torch, path, ids_list, dev, stream):
        import numpy as np
        self.lib, self.torch, self.dev = lib, torch, dev
        self.model = bertpy.BertModel(path, lib=lib)
        ctx = self.model.ctx
        B = len(ids_list)
        lens = [len(x) for x in ids_list]
        self.B, self.T, self.L = B, sum(lens), max(lens)
        self.ids = torch.from_numpy(np.concatenate(ids_list).astype(np.int32)).to(dev)
        self.cu = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)).to(dev)
        self.out = torch.empty((B, self.model.n_embd), dtype=torch.float32, device=dev)
        assert lib.bertx_reserve(ctx, 0, self.T, B) == 0
        self.sp = ctypes.c_void_p(stream.cuda_stream)
        self.args = (ctx, 0, ctypes.c_void_p(self.ids.data_ptr()), ctypes.c_void_p(self.cu.data_ptr()), B, self.L,
                     self.T, ctypes.c_void_p(self.out.data_ptr()), self.sp)

    def step(self):
        rc = self.lib.bertx_forward_device(*self.args)
        if rc != 0:
            raise RuntimeError(f"bertx_forward_device failed: {rc}")

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    def check(self):
        import numpy as np
        e = self.out.float().cpu().numpy()
        assert np.all(np.isfinite(e)) and np.allclose(np.linalg.norm(e, axis=1), 1.0, atol=1e-3), "bad embeddings"
        return e

    def kernel_pass(self, steps):
        """K eager forwards with a HIP event pair around every kernel on the
        launch stream; returns the per-class stats."""
        ctx = self.model.ctx
        self.lib.bertx_set_profiling(ctx, 1)
        self.lib.bertx_reset_stats(ctx)
        t = timed_steps(self.step, steps, self.sync)
        self.lib.bertx_set_profiling(ctx, 0)
        return t, self.model.kernel_stats()


def ensure_model(bertpy, model_dir, arch, ftype, seed):
    os.makedirs(model_dir, exist_ok=True)
    path = os.path.join(model_dir, f"{arch}-{ftype}-seed{seed}.bin")
    if not os.path.exists(path):
        bertpy.synthetic_model(path + ".part", arch, ftype, seed=seed)
        os.replace(path + ".part", path)
    return path


def dominant(stats):
    """(class name, avg launch seconds, work per launch, work is FLOP) of the class with the most time."""
    live = [s for s in stats if s["launches"]]
    if not live:
        return None
    dom = max(live, key=lambda s: s["ms"])
    return dom["name"], dom["ms"] / dom["launches"] * 1e-3, dom["work"] / dom["launches"], dom["work_is_flops"]


# --------------------------------------------------------------------------
# this run's HBM counters (north_star: "rocprof reports achieved HBM GB/s")
# --------------------------------------------------------------------------
PROBE_BIN = os.path.join(ROOT, "build", "bin", "bert_probe")


def kernel_class(name, state):
    """bench kernel class of a rocprofv3 kernel name (mangled or demangled); the two
    residual GEMMs of a layer (O-proj, FFN-down) share a form and alternate in
    dispatch order (state counts them)."""
    m = re.search(r"gemm[a-z0-9]*_kernelILi(\d+)ELi(\d+)E", name) or \
        re.search(r"gemm[a-z0-9]*_kernel<(\d+), (\d+)", name)
    if m:
        epi = int(m.group(2))
        if epi == 0:
            return "gemm_qkv"
        if epi == 1:
            return "gemm_ffn_up"
        state["res"] = state.get("res", 0) + 1
        return "gemm_attn_out" if state["res"] % 2 == 1 else "gemm_ffn_down"
    for key, cls in (("attention", "attention"), ("ln_stats", "ln_stats"), ("embed_ln", "embed_ln"),
                     ("pool_", "pool_l2")):
        if key in name:
            return cls
    return None


def pmc_pass(model_path, B, L, counter, steps, warmup, timeout_s, device):
    """One rocprofv3 counter pass over bert_probe (eager launches, so every kernel is
    its own dispatch); returns [(class, KiB)] of the last `steps` forwards in dispatch
    order, or raises."""
    rp = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    out = tempfile.mkdtemp(prefix="bench_pmc_", dir="/tmp")
    try:
        env = dict(os.environ, BERT_GRAPHS="0", BERT_DEVICES=str(device), TMPDIR="/tmp")
        if os.environ.get("BERT_LIB"):
            # A/B runs against another build: the probe's RUNPATH ($ORIGIN/..) would
            # load build/libbert.so; LD_LIBRARY_PATH is searched before a RUNPATH
            lp = os.path.dirname(os.path.abspath(os.environ["BERT_LIB"]))
            env["LD_LIBRARY_PATH"] = lp + (":" + env["LD_LIBRARY_PATH"] if env.get("LD_LIBRARY_PATH") else "")
        cmd = ["timeout", "-s", "KILL", str(timeout_s), rp, "--pmc", counter, "--output-format", "csv",
               "-d", out, "-o", "pmc", "--", PROBE_BIN, model_path, str(B), str(L), str(steps), str(warmup)]
        r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                           timeout=timeout_s + 30)
        if r.returncode != 0:
            raise RuntimeError(f"rocprofv3 --pmc {counter} rc {r.returncode}: "
                               + r.stdout.decode(errors="replace")[-300:])
        files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            raise RuntimeError(f"no counter_collection.csv from rocprofv3 --pmc {counter}")
        rows = [x for x in csv.DictReader(open(files[0])) if x["Counter_Name"] == counter]
        rows.sort(key=lambda x: int(x["Dispatch_Id"]))
        st, seq = {}, []
        for x in rows:
            c = kernel_class(x["Kernel_Name"], st)
            if c:
                seq.append((c, float(x["Counter_Value"])))
        per_fwd = len(seq) // (steps + warmup)
        if per_fwd == 0 or per_fwd * (steps + warmup) != len(seq):
            raise RuntimeError(f"{len(seq)} kernel dispatches for {steps + warmup} forwards")
        return seq[-steps * per_fwd:]
    finally:
        shutil.rmtree(out, ignore_errors=True)


def under_profiler(env=None):
    """True when this process already runs under a profiler (rocprofv3 preloads its
    tool library and exports ROCP*/ROCPROF* variables into the profiled program).
    Starting rocprofv3 (a #!/usr/bin/env python3 script) from such a process is an
    exec from a GPU-initialised process tree, which this pool refuses."""
    env = os.environ if env is None else env
    pre = env.get("LD_PRELOAD", "")
    if re.search(r"roctracer|rocprof|rocprofiler|libroctx|rocm_sdk", pre, re.I):
        return True
    return any(k.startswith(("ROCP_", "ROCPROF", "ROCPROFILER", "ROCTX", "ROCP_TOOL")) for k in env)


def pmc_live(model_path, B, L, device=0, steps=2, warmup=1, timeout_s=120):
    """This run's HBM-side traffic of one forward of B x L tokens, per kernel class:
    2 x FETCH_SIZE + WRITE_SIZE (KiB -> B; gfx950 FETCH_SIZE counts half the bytes of
    16-B-per-lane reads, MI355X_MICROARCH.md "HBM"), from two rocprofv3 --pmc passes
    (the two counters cannot share a pass) over build/bin/bert_probe.  Infinity-Cache
    hits are included, so this is an upper bound on DRAM bytes.  Under a profiler
    (under_profiler) nothing is started: the result says so."""
    if under_profiler():
        return {"skipped": "under a profiler (rocprofv3 preload in this process): no nested rocprofv3 passes"}
    t0 = time.perf_counter()
    fetch = pmc_pass(model_path, B, L, "FETCH_SIZE", steps, warmup, timeout_s, device)
    write = pmc_pass(model_path, B, L, "WRITE_SIZE", steps, warmup, timeout_s, device)
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for c, v in fetch:
        agg[c][0] += 2.0 * v * 1024 / steps
        agg[c][2] += 1
    for c, v in write:
        agg[c][1] += v * 1024 / steps
    per_class = {}
    for c, (fb, wb, n) in sorted(agg.items()):
        launches = n / steps
        per_class[c] = {"launches_per_forward": launches, "bytes_per_launch": int((fb + wb) / launches),
                        "fetch_bytes_per_forward": int(fb), "write_bytes_per_forward": int(wb)}
    total = int(sum(v[0] + v[1] for v in agg.values()))
    return {"bytes_per_forward": total, "per_class": per_class, "forwards_counted": steps,
            "source": "this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over build/bin/bert_probe "
                      "(eager launches of the same kernels), 2 x FETCH_SIZE + WRITE_SIZE per MI355X_MICROARCH.md",
            "pmc_seconds": round(time.perf_counter() - t0, 1)}


def probes(lib, bertpy, torch, a, dev, stream, q4_path):
    """BASELINE.json north_star: 'rocprof reports achieved HBM GB/s on the q4_0 path and
    MFMA utilisation on the f16 path against gfx950 peak'.  Two probes, each timed
    like the headline (graph replay between syncs, then an evented pass):
      f16_mfma: C2 = all-MiniLM-L6-v2 f16, L 128, B 32 -- sentences/s and the
        dominant kernel's achieved TFLOP/s against the 2.5 PF dense f16 peak;
      q4_0_hbm: bge-base q4_0, B 1, L 32 (SURVEY §8d's bandwidth-bound probe, AI ~40)
        -- forward latency and algorithmic bytes (weights at stored width + rows +
        ids + output) / latency against 8 TB/s, and this run's counter bytes (pmc_live)
        / latency beside it.  The probe always builds bge-base-en-v1.5 q4_0, whatever
        --arch/--ftype the headline runs;
      c4_shard / c5_ragged: BASELINE.json's C4 at one GPU's share and C5 -- sentences/s,
        tokens/s and the dominant kernel."""
    out = {}
    steps = max(a.steps, 20)
    # C2
    hp = bertpy.ARCHS["all-MiniLM-L6-v2"]
    p2 = ensure_model(bertpy, a.model_dir, "all-MiniLM-L6-v2", "f16", a.seed)
    f = DeviceForward(lib, bertpy, torch, p2, bertpy.synthetic_ids(32, 128, hp["n_vocab"], seed=7), dev, stream)
    for _ in range(3):
        f.step()
    f.sync()
    f.check()
    el = timed_steps(f.step, steps, f.sync)
    _, st = f.kernel_pass(steps)
    name, avg_s, work, is_flops = dominant(st)
    ach = work / avg_s / 1e12
    out["f16_mfma"] = {"workload": "C2 all-MiniLM-L6-v2 f16, L 128, B 32 (bertx_forward_device)",
                       "sentences_per_s": round(32 * steps / el, 1), "ms_per_batch": round(el / steps * 1e3, 4),
                       "dominant_kernel": name, "avg_launch_us": round(avg_s * 1e6, 2),
                       "achieved_tflops": round(ach, 1), "peak_tflops": MFMA_F16_PEAK_TFLOPS,
                       "mfma_frac": round(ach / MFMA_F16_PEAK_TFLOPS, 4),
                       "step_tflops": round(32 * flop_per_sentence(hp, 128) * steps / el / 1e12, 1),
                       "kernel_avg_us": {s["name"]: round(s["ms"] * 1e3 / s["launches"], 2)
                                         for s in st if s["launches"]}}
    if not a.no_pmc:
        try:
            pm = pmc_live(p2, 32, 128, device=int(os.environ.get("LOCAL_RANK", "0")))
            if "bytes_per_forward" in pm:
                pm["gbps_at_measured_step"] = round(pm["bytes_per_forward"] / (el / steps) / 1e9, 1)
            out["f16_mfma"]["pmc"] = pm
        except Exception as ex:   # a report, never the metric
            out["f16_mfma"]["pmc"] = {"error": str(ex)}
    del f
    # bandwidth probe: bge-base q4_0, one sentence of 32 tokens
    hp = bertpy.ARCHS["bge-base-en-v1.5"]
    q4_path = ensure_model(bertpy, a.model_dir, "bge-base-en-v1.5", "q4_0", a.seed)
    f = DeviceForward(lib, bertpy, torch, q4_path, bertpy.synthetic_ids(1, 32, hp["n_vocab"], seed=7), dev, stream)
    for _ in range(3):
        f.step()
    f.sync()
    f.check()
    steps_b = max(200, steps)
    el = timed_steps(f.step, steps_b, f.sync)
    lat = el / steps_b
    by = algorithmic_bytes(hp, "q4_0", 1, 32)
    _, st = f.kernel_pass(steps_b)
    launches = sum(s["launches"] for s in st) / steps_b
    kern_s = sum(s["ms"] for s in st) * 1e-3 / steps_b
    out["q4_0_hbm"] = {"workload": "bge-base-en-v1.5 q4_0, B 1, L 32 (bertx_forward_device)",
                       "latency_us": round(lat * 1e6, 1), "algorithmic_bytes": int(by),
                       "achieved_gbps": round(by / lat / 1e9, 1), "peak_gbps": HBM_PEAK_GBPS,
                       "hbm_frac": round(by / lat / 1e9 / HBM_PEAK_GBPS, 4),
                       "kernels_per_forward": launches, "sum_kernel_us": round(kern_s * 1e6, 1),
                       "kernel_avg_us": {s["name"]: round(s["ms"] * 1e3 / s["launches"], 2)
                                         for s in st if s["launches"]}}
    if not a.no_pmc:
        try:
            pm = pmc_live(q4_path, 1, 32, device=int(os.environ.get("LOCAL_RANK", "0")), steps=3)
            if "bytes_per_forward" in pm:
                gbps = pm["bytes_per_forward"] / lat / 1e9
                pm.update({"counter_gbps": round(gbps, 2), "counter_hbm_frac": round(gbps / HBM_PEAK_GBPS, 5)})
            out["q4_0_hbm"]["pmc"] = pm
        except Exception as ex:
            out["q4_0_hbm"]["pmc"] = {"error": str(ex)}
    del f
    # C1 (BASELINE.json configs[0]): all-MiniLM-L6-v2 f32, one sentence of 32 tokens --
    # the reference's CPU plumbing case; here on the f32 chain (f32 activations x f32
    # weights, f32.hip).  The CPU side of C1 is timed in the cpu_baseline leg.
    try:
        hp = bertpy.ARCHS["all-MiniLM-L6-v2"]
        p1 = ensure_model(bertpy, a.model_dir, "all-MiniLM-L6-v2", "f32", a.seed)
        f = DeviceForward(lib, bertpy, torch, p1, bertpy.synthetic_ids(1, 32, hp["n_vocab"], seed=7), dev, stream)
        for _ in range(3):
            f.step()
        f.sync()
        f.check()
        n1 = max(200, steps)
        el = timed_steps(f.step, n1, f.sync)
        _, st = f.kernel_pass(n1)
        out["c1_f32"] = {"workload": "C1 all-MiniLM-L6-v2 f32, B 1, L 32 (bertx_forward_device, the f32 chain)",
                         "latency_us": round(el / n1 * 1e6, 1), "sentences_per_s": round(n1 / el, 1),
                         "kernel_avg_us": {s["name"]: round(s["ms"] * 1e3 / s["launches"], 2)
                                           for s in st if s["launches"]}}
        del f
    except Exception as ex:   # a probe is a report, never the metric
        out["c1_f32"] = {"error": str(ex)}
    # the other two GPU configs of BASELINE.json at one GPU's share: C4 (bge-large q4_1,
    # L 512, 256 sentences over 8 GPUs = 32 per GPU: the replicas-only multi-GPU
    # path runs exactly this per GPU) and C5 (bge-base-zh q8_0, 128 ragged sentences)
    import numpy as np
    rng = np.random.default_rng(11)
    for key, arch, ftype, lens, what in (
            ("c4_shard", "bge-large-en-v1.5", "q4_1", [512] * 32,
             "C4 per GPU: bge-large-en-v1.5 q4_1, L 512, 32 sentences (256 over 8 GPUs as replicas)"),
            ("c5_ragged", "bge-base-zh-v1.5", "q8_0", [int(x) for x in rng.integers(16, 513, 128)],
             "C5: bge-base-zh-v1.5 q8_0, 128 sentences, lengths uniform in [16, 512] (seed 11)")):
        try:
            hp = bertpy.ARCHS[arch]
            pth = ensure_model(bertpy, a.model_dir, arch, ftype, a.seed)
            f = DeviceForward(lib, bertpy, torch, pth, bertpy.synthetic_ids(len(lens), lens, hp["n_vocab"], seed=7),
                              dev, stream)
            for _ in range(3):
                f.step()
            f.sync()
            f.check()
            n = max(5, min(steps, 20))
            el = timed_steps(f.step, n, f.sync)
            _, st = f.kernel_pass(n)
            name, avg_s, work, is_flops = dominant(st)
            rec = {"workload": what, "sentences_per_s": round(len(lens) * n / el, 1),
                   "tokens_per_s": round(sum(lens) * n / el, 0), "ms_per_batch": round(el / n * 1e3, 4),
                   "dominant_kernel": name, "avg_launch_us": round(avg_s * 1e6, 2)}
            if is_flops:
                ach = work / avg_s / 1e12
                rec.update({"achieved_tflops": round(ach, 1), "mfma_frac": round(ach / MFMA_F16_PEAK_TFLOPS, 4)})
            out[key] = rec
            del f
        except Exception as ex:   # a probe is a report, never the metric
            out[key] = {"error": str(ex)}
    return out


def all_ranks_ok(ok, dist, red_dev):
    """True on every rank iff `ok` is True on every rank (a MIN all-reduce; no
    collective without torch.distributed)."""
    if dist is None:
        return ok
    import torch
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=red_dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def library_path(model, ids_list, steps, dist, red_dev):
    """The reference Python client's path (examples/sample_dylib.py -> bert_forward_batch):
    host int32 token arrays in, host float32 rows out -- staging copy, H2D, forward,
    D2H and the copy into the caller's rows all inside the timed region; synchronous
    calls, K of them between barriers, max over ranks."""
    for _ in range(2):
        model.forward_batch(ids_list)
    el = timed_steps(lambda: model.forward_batch(ids_list), steps, lambda: None, dist, red_dev)
    return el


def encode_path(lib, model, ids_list, steps, dist, red_dev, ref):
    """SURVEY §8d end-to-end: the same batch as TEXT through bert_encode_batch
    (bert.cpp:1374-1444, the entry examples/sample_dylib.py:57-59 calls): tokenize
    on the library's pool, sort and chunk, stage, H2D, forward, D2H into the
    caller's rows.  Each text is the bench's ids as words of the synthetic vocab
    ('w<i>' = id 104 + i, bertpy.synthetic_vocab), so it tokenizes to exactly those
    512 ids.  Tokenizer threads = this job's CPU share.  Also times the tokenizer
    stage alone (bertx_tokenize_batch, bert_encode_batch's first stage) to report
    its share of the call."""
    import numpy as np
    # rank-local preparation, then every rank agrees before the collectives of the
    # timed region: a rank that failed here (e.g. a tokenize mismatch) must not leave
    # the others waiting in its barrier
    err = None
    try:
        texts = [" ".join("w%d" % (int(t) - 104) for t in ids[1:-1]).encode() for ids in ids_list]
        toks, n = model.tokenize(texts[0])
        if n != len(ids_list[0]) or toks != [int(x) for x in ids_list[0]]:
            raise RuntimeError("encode texts do not tokenize to the bench ids")
        share = len(os.sched_getaffinity(0))
        n_thr = max(1, min(share, int(os.environ.get("OMP_NUM_THREADS", share))))
        B, d = len(texts), model.n_embd
        out = np.zeros((B, d), np.float32)
        rows = (out.ctypes.data + out.strides[0] * np.arange(B, dtype=np.uintp)).astype(np.uintp)
        rows_p = rows.ctypes.data_as(ctypes.POINTER(ctypes.POINTER(ctypes.c_float)))
        carr = (ctypes.c_char_p * B)(*texts)

        def call():
            lib.bert_encode_batch(model.ctx, n_thr, B, B, carr, rows_p)
        for _ in range(2):
            call()
    except Exception as ex:   # noqa: BLE001 -- agreed on below, then reported
        err = ex
    if not all_ranks_ok(err is None, dist, red_dev):
        raise RuntimeError(f"encode leg skipped on every rank ({err or 'another rank failed its preparation'})")
    same = bool(ref is not None and np.array_equal(out, ref))
    cos = float(np.min(np.sum(out * ref, axis=1))) if ref is not None else None
    el = timed_steps(call, steps, lambda: None, dist, red_dev)
    nmax = model.n_max_tokens
    ids_buf = np.zeros((B, nmax), np.int32)
    lens = np.zeros(B, np.int32)
    t0 = time.perf_counter()
    for _ in range(steps):
        if lib.bertx_tokenize_batch(model.ctx, n_thr, B, carr, nmax, ids_buf.ctypes.data, lens.ctypes.data) != 0:
            raise RuntimeError("bertx_tokenize_batch failed")
    tok_s = (time.perf_counter() - t0) / steps
    world = dist.get_world_size() if dist is not None else 1
    return {"value": round(B * world * steps / el, 2), "unit": "sentences/s", "ms_per_step": round(el / steps * 1e3, 4),
            "tokenizer_ms": round(tok_s * 1e3, 4), "tokenizer_share": round(tok_s / (el / steps), 4),
            "tokenizer_threads": n_thr, "bitwise_equal_to_device_path": same, "min_cosine_vs_device_path": cos,
            "workload": f"the same {B} sentences per GPU as text ({len(ids_list[0])} tokens each, single-token "
                        "vocab words) through bert_encode_batch(n_batch_size = n_inputs): tokenization, staging, "
                        "H2D, forward, D2H inside the timed region, one context per rank"}


def run_inproc(a):
    """--inproc: ONE process drives a.gpus GPUs through the library's own multi-GPU
    path (bert_abi.cpp run_forward: sentences split over the context's GPUs by FLOP
    cost, one host thread + stream + weight replica per GPU, no collectives) -- what
    ctypes and server callers get from bert_forward_batch.  Prints one JSON line."""
    if "BERT_DEVICES" not in os.environ:
        os.environ["BERT_DEVICES"] = ",".join(str(i) for i in range(a.gpus))
    import numpy as np
    import bertpy
    hp = bertpy.ARCHS[a.inproc_arch]
    path = ensure_model(bertpy, a.model_dir, a.inproc_arch, a.inproc_ftype, a.seed)
    m = bertpy.BertModel(path)
    nd = m.lib.bertx_num_devices(m.ctx)
    ids = bertpy.synthetic_ids(a.inproc_batch, a.seq, hp["n_vocab"], seed=7)
    for _ in range(max(a.warmup, 1)):
        e = m.forward_batch(ids)
    assert np.all(np.isfinite(e)) and np.allclose(np.linalg.norm(e, axis=1), 1.0, atol=1e-3)
    el = timed_steps(lambda: m.forward_batch(ids), a.steps, lambda: None)
    per = m.device_last_call()
    busy = [p[0] for p in per if p[1] > 0]
    flop = a.inproc_batch * flop_per_sentence(hp, a.seq)
    res = {"metric": f"sentences/sec, {a.inproc_arch} {a.inproc_ftype} seq{a.seq} batch{a.inproc_batch}, "
                     "library path (bert_forward_batch, host buffers, in-process multi-GPU)",
           "value": round(a.inproc_batch * a.steps / el, 2), "unit": "sentences/s", "n_gpus": nd,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3),
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f16",
           "data": "synthetic (random-init weights, seeded token ids)",
           "config": {"workload": f"{a.inproc_arch} {a.inproc_ftype} seq_len {a.seq}, {a.inproc_batch} sentences "
                                  f"split over {nd} GPU replicas by bert_forward_batch",
                      "global_batch": a.inproc_batch, "seq_len": a.seq, "weights": a.inproc_ftype,
                      "devices": os.environ["BERT_DEVICES"], "parallelism": f"in-process replicas x{nd}"},
           "tflops": round(flop * a.steps / el / 1e12, 1),
           "per_device_last_call": [{"slot": i, "wall_ms": round(p[0], 3), "sentences": p[1], "tokens": p[2]}
                                    for i, p in enumerate(per)],
           "balance_max_over_min_wall": round(max(busy) / min(busy), 3) if busy else None}
    print(json.dumps(res), flush=True)


def flop_per_sentence(hp, L):
    d, f, nl = hp["n_embd"], hp["n_intermediate"], hp["n_layer"]
    return nl * (2 * L * (4 * d * d + 2 * d * f) + 4 * L * L * d)


class DryForward:
    """--dry-step: a CPU stand-in for DeviceForward (no library, no GPU) so the
    multi-rank launch, timing and reporting skeleton runs under gloo on a CPU host."""

    def __init__(self, B, d=768):
        self.B, self.d, self.model = B, d, None

    def step(self):
        time.sleep(0.002)

    def sync(self):
        pass

    def check(self):
        return None


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ and not a.inproc:
        # a plain `python bench.py --gpus N`: start the N ranks (before any GPU call here)
        sys.exit(launch_ranks(a))
    rank, world, local = dist_env()
    if a.inproc:
        assert world == 1, "--inproc runs in one process"
        run_inproc(a)
        return
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE {world}: every GPU is one rank "
                         "(run `python bench.py --gpus N`, or torchrun with --nproc-per-node N)")
    # BENCH_SHARED_DEVICE=1 (rehearsal of the N-rank path on a one-GPU box): every
    # rank drives GPU 0 and the timing collectives go over gloo (RCCL does not run
    # two ranks on one GPU); the per-rank rates then share that GPU
    shared = os.environ.get("BENCH_SHARED_DEVICE", "0") == "1" and world > 1
    if shared:
        local = 0
    os.environ["BERT_DEVICES"] = str(local)
    import numpy as np
    import torch
    import bertpy

    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = "gloo" if (a.dry_step or shared) else ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    elif not a.dry_step:
        torch.cuda.set_device(local)

    hp = bertpy.ARCHS[a.arch]
    B, L = a.batch, a.seq
    ids_list = bertpy.synthetic_ids(B, L, hp["n_vocab"], seed=7 + rank)
    path = os.path.join(a.model_dir, f"{a.arch}-{a.ftype}-seed{a.seed}.bin")
    if a.dry_step:
        fwd = DryForward(B, hp["n_embd"])
        dev, stream, lib, model = None, None, None, None
        sync = fwd.sync
    else:
        if rank == 0:
            path = ensure_model(bertpy, a.model_dir, a.arch, a.ftype, a.seed)
        if dist is not None:
            dist.barrier()
        lib = bertpy.load_lib()
        dev = torch.device("cuda", local)
        # a non-default stream: the library captures the forward into a HIP graph
        # (capture is impossible on the legacy null stream)
        stream = torch.cuda.Stream(dev)
        torch.cuda.set_stream(stream)
        fwd = DeviceForward(lib, bertpy, torch, path, ids_list, dev, stream)
        model = fwd.model
        sync = lambda: torch.cuda.synchronize(dev)
    step = fwd.step

    for _ in range(a.warmup):
        step()
    sync()
    e = fwd.check()

    red_dev = dev if (dist is not None and dist.get_backend() == "nccl") else "cpu"
    # timed region (the metric): graph replay of the forward, no per-kernel events
    if lib is not None:
        lib.bertx_set_profiling(model.ctx, 0)
    rank_elapsed = []
    elapsed = timed_steps(step, a.steps, sync, dist, red_dev, per_rank=rank_elapsed)
    # roofline pass: the same K steps again, launched eagerly with a HIP event
    # pair around every kernel on the launch stream (per-kernel averages)
    stats = []
    profiled = lib is not None and not a.no_profile
    if profiled:
        lib.bertx_set_profiling(model.ctx, 1)
        lib.bertx_reset_stats(model.ctx)
        prof_elapsed = timed_steps(step, a.steps, sync, dist, red_dev)
        lib.bertx_set_profiling(model.ctx, 0)
        stats = model.kernel_stats()

    ms_per_step = elapsed / a.steps * 1e3
    value = B * world * a.steps / elapsed
    lib_el = None
    if lib is not None and not a.no_library:
        lib_el = library_path(model, ids_list, a.steps, dist, red_dev)
    enc = None
    if lib is not None and not a.no_encode:
        try:
            enc = encode_path(lib, model, ids_list, a.steps, dist, red_dev, e)
        except Exception as ex:   # a report, never the metric
            enc = {"error": str(ex)}

    roofline = None
    kernels = {}
    for s in stats:
        if s["launches"]:
            kernels[s["name"]] = {"launches": s["launches"], "avg_us": s["ms"] / s["launches"] * 1e3,
                                  "share": 0.0}
    tot_ms = sum(s["ms"] for s in stats) or 1.0
    for s in stats:
        if s["launches"]:
            kernels[s["name"]]["share"] = round(s["ms"] / tot_ms, 4)
    if stats and profiled:
        dom = max(stats, key=lambda s: s["ms"])
        if dom["launches"]:
            avg_s = dom["ms"] / dom["launches"] * 1e-3
            per_launch = dom["work"] / dom["launches"]
            if dom["work_is_flops"]:
                ach = per_launch / avg_s / 1e12
                roofline = {"kernel": dom["name"], "bound": "mfma", "achieved": round(ach, 2),
                            "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / MFMA_F16_PEAK_TFLOPS, 4),
                            "work_per_launch": per_launch, "avg_launch_us": round(avg_s * 1e6, 2), "traffic": None}
            else:
                ach = per_launch / avg_s / 1e9
                roofline = {"kernel": dom["name"], "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS,
                            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": None}

    # this run's HBM counters for the headline workload (rank 0 of a single-process
    # run: two rocprofv3 --pmc passes over build/bin/bert_probe on the same model)
    pm = None
    if rank == 0 and world == 1 and not a.no_pmc and lib is not None:
        try:
            pm = pmc_live(path, B, L, device=local)
        except Exception as ex:   # a report, never the metric
            pm = {"error": str(ex)}
    if roofline:
        if pm and "per_class" in pm and roofline["kernel"] in pm["per_class"]:
            roofline["traffic"] = pm["per_class"][roofline["kernel"]]["bytes_per_launch"]
            roofline["traffic_source"] = "this run (rocprofv3 PMC, 2 x FETCH_SIZE + WRITE_SIZE per launch)"
        else:
            rec = os.path.join(ROOT, "profiles", "pmc_traffic.json")
            if os.path.exists(rec):
                try:
                    with open(rec) as f:
                        tr = json.load(f).get(roofline["kernel"])
                    if tr is not None:
                        roofline["traffic"] = tr
                        roofline["traffic_source"] = "recorded: profiles/pmc_traffic.json (an earlier PMC session)"
                except Exception:
                    pass

    alg_bytes = algorithmic_bytes(hp, a.ftype, B, L)
    res = {
        "metric": "sentences/sec + HBM GB/s, bge-base-en-v1.5 q4_0 seq512 batch64, 1/2/4/8 GPU",
        "value": round(value, 2), "unit": "sentences/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f16",
        "data": "dry-step CPU stub (no forward; launch/timing skeleton only)" if a.dry_step
                else "synthetic (random-init weights, seeded token ids)",
        "config": {"workload": f"{a.arch} {a.ftype} seq_len {L}, {B} sentences per GPU: bertx_forward_device on "
                               f"HBM-resident token ids (the bert_forward_batch graph without its H2D/D2H)",
                   "batch_per_gpu": B, "global_batch": B * world, "seq_len": L, "weights": a.ftype,
                   "parallelism": f"replicas x{world} (no collectives)"},
        # compulsory bytes (weights at stored width, gathered rows, ids, output) per
        # step / step time: at C3 the path is MFMA-bound (AI ~1e5 FLOP/B), so this is
        # NOT an HBM-roofline figure -- see probes.q4_0_hbm and roofline.traffic
        "compulsory_gbps": round(alg_bytes / (ms_per_step * 1e-3) / 1e9, 2),
        "timing": "value: K graph-replayed forwards (no events); roofline/kernels: a second pass of K eager "
                  "forwards with HIP events around every kernel"
                  + (f" ({prof_elapsed / a.steps * 1e3:.3f} ms/step)" if profiled else ""),
        "roofline": roofline,
        "kernels": kernels,
        # every rank's own rate over the same timed region (value uses the max time)
        "per_rank": [{"rank": r, "sentences_per_s": round(B * a.steps / t, 2), "ms_per_step": round(t / a.steps * 1e3, 4)}
                     for r, t in enumerate(rank_elapsed)],
    }
    if shared:
        res["shared_device_rehearsal"] = f"BENCH_SHARED_DEVICE=1: all {world} ranks on GPU 0 (gloo timing collectives)"
    # measured HBM traffic of the step: this run's PMC bytes of one forward over the
    # graph-replayed step time
    if pm is not None:
        if "bytes_per_forward" in pm:
            gb = pm["bytes_per_forward"] / (ms_per_step * 1e-3) / 1e9
            res["hbm"] = {"bytes_per_step": pm["bytes_per_forward"], "gbps": round(gb, 1), "peak_gbps": HBM_PEAK_GBPS,
                          "frac": round(gb / HBM_PEAK_GBPS, 4), "per_class": pm["per_class"], "source": pm["source"],
                          "pmc_seconds": pm["pmc_seconds"]}
        else:
            res["hbm"] = pm
    if lib_el is not None:
        res["library_path"] = {"value": round(B * world * a.steps / lib_el, 2), "unit": "sentences/s",
                               "ms_per_step": round(lib_el / a.steps * 1e3, 4),
                               "workload": "the same batch per GPU through bert_forward_batch from host int32 "
                                           "arrays into host float rows (the ctypes client's path: staging, "
                                           "H2D, forward, D2H inside the timed region), one context per rank"}

    if enc is not None:
        res["encode_path"] = enc
    if rank == 0 and world == 1 and not a.no_cpu_baseline and lib is not None:
        try:
            import oracle_lib
            # the GPU box gives one GPU's job a 16-CPU share (OMP_NUM_THREADS=16 there;
            # os.cpu_count() shows the whole machine): use every core of that share
            share = len(os.sched_getaffinity(0))
            n_thr = max(1, min(share, int(os.environ.get("OMP_NUM_THREADS", share))))
            orc = oracle_lib.Oracle(path)
            sample = [x for x in ids_list[: a.cpu_baseline_sentences]]
            c0 = time.perf_counter()
            emb_cpu = orc.forward_batch(sample, n_threads=n_thr)
            c1 = time.perf_counter()
            cos = float(np.min(np.sum(emb_cpu * e[: len(sample)], axis=1)))
            res["cpu_baseline"] = {"value": round(len(sample) / (c1 - c0), 4), "unit": "sentences/s",
                                   "cores": n_thr, "kind": "port",
                                   "sample": f"{len(sample)} of the {B} sentences (L={L}) through the C oracle "
                                             f"(oracle/bert_oracle.c, ggml-era q8 activation path) on {n_thr} "
                                             f"threads = this job's CPU share ({share} CPUs visible, "
                                             f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}), "
                                             f"{c1 - c0:.1f} s",
                                   "gpu_vs_cpu_min_cosine": round(cos, 6)}
        except Exception as ex:  # the baseline is a report, never the product
            res["cpu_baseline"] = {"value": None, "error": str(ex)}
        if not a.no_probes:
            # C1 (BASELINE.json configs[0], the reference's CPU case): all-MiniLM-L6-v2
            # f32, one 32-token sentence, the oracle on this job's CPU share against the
            # GPU's f32 chain through bert_forward_batch (the probes time the GPU side)
            try:
                import oracle_lib
                share = len(os.sched_getaffinity(0))
                n_thr = max(1, min(share, int(os.environ.get("OMP_NUM_THREADS", share))))
                hp1 = bertpy.ARCHS["all-MiniLM-L6-v2"]
                p1 = ensure_model(bertpy, a.model_dir, "all-MiniLM-L6-v2", "f32", a.seed)
                ids1 = bertpy.synthetic_ids(1, 32, hp1["n_vocab"], seed=7)
                g1 = bertpy.BertModel(p1, lib=lib).forward_batch(ids1)
                o1 = oracle_lib.Oracle(p1)
                o1.forward_batch(ids1, n_threads=n_thr)          # warm (page-in, tables)
                reps = 20
                c0 = time.perf_counter()
                for _ in range(reps):
                    c1e = o1.forward_batch(ids1, n_threads=n_thr)
                c1 = time.perf_counter()
                res["cpu_baseline"]["c1"] = {
                    "workload": "C1 all-MiniLM-L6-v2 f32, B 1, L 32: the C oracle (f32 x f32, as the reference's "
                                "f32 path) on this job's CPU share",
                    "cpu_ms_per_sentence": round((c1 - c0) / reps * 1e3, 3), "cores": n_thr,
                    "gpu_vs_cpu_cosine": round(float(np.sum(g1[0] * c1e[0])), 9)}
            except Exception as ex:   # a report, never the product
                res["cpu_baseline"]["c1"] = {"error": str(ex)}

    if rank == 0 and world == 1 and not a.no_probes and lib is not None:
        try:
            res["probes"] = probes(lib, bertpy, torch, a, dev, stream, path)
        except Exception as ex:   # a probe is a report, never the metric
            res["probes"] = {"error": str(ex)}

    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Pi0 training throughput (+ action-chunk inference latency) on MI355X.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json metric, configs[1]/[2]): bridge-shaped synthetic batch
(256 image + 20 text + 1 proprio + 4 action tokens), full Pi0 (SigLIP-So400m +
Gemma-2B + 0.3B action expert, random-init weights), bf16, flow-matching
forward + backward + grad-norm clip + AdamW (8-bit blockwise state, the reference's
bnb AdamW8bit) over 2.6B trained parameters.
One step = one optimizer update at global batch 1024 (= N GPUs x micro-batch x
accumulation); with N GPUs the grads are all-reduced over RCCL, overlapped
with the last micro-batch's backward.  ``value`` = samples/s of the whole job.
Also reported: bf16 action-chunk inference latency (B=1, hipGraph replay),
the dominant kernel's roofline (live HIP-event timing of the vlm GeGLU GEMM),
and the CPU restatement (oracle/) timed on this host.
"""

from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0  # dense MFMA bf16 (MI355X_MICROARCH.md)
TRAIN_FLOP_PER_SAMPLE = 3.812e12  # SURVEY 8(d), FlopCounterMode on the reference
PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
PEAK_FP8_TFLOPS = 5000.0  # dense MFMA e4m3 (MI355X_MICROARCH.md)
C5_PREFILL_FLOP = 3.711e12  # 3 images + 20 text + 1 proprio prefill (FlopCounterMode on the reference)
INFER_BYTES = 11.5e9  # B=1 action chunk, weights streamed + KV reads


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def synthetic_batch(model, B, device, gen):
    d = model._engine().d
    ids = torch.full((B, d.P), 0, dtype=torch.int64)
    ids[:, : d.n_img] = d.image_token
    ids[:, d.n_img] = 2
    ids[:, d.n_img + 1 : d.P - 1] = torch.randint(3, 256000, (B, d.P - d.n_img - 2), generator=gen)
    ids[:, d.P - 1] = 108
    am = (ids != 0).long()
    mask, vpos, ppos, apos = model.build_causal_mask_and_position_ids(am, torch.bfloat16)
    u = torch.rand(B, generator=gen)
    t = 0.999 * (1 - u.pow(1 / 1.5))  # Beta(1.5, 1) flipped (train.py:239-247)
    return dict(
        input_ids=ids.to(device), pixel_values=(torch.rand(B, 3, d.img, d.img, generator=gen) * 2 - 1).to(device, torch.bfloat16),
        causal_mask=mask.to(device), vlm_position_ids=vpos.to(device), proprio_position_ids=ppos.to(device),
        action_position_ids=apos.to(device), proprios=(torch.rand(B, d.C, d.Pd, generator=gen) * 2 - 1).to(device),
        actions=(torch.rand(B, d.H, d.A, generator=gen) * 2 - 1).to(device), t=t.to(device),
    )


def pmc_traffic(kname, shape):
    """HBM bytes per launch of the dominant kernel from the committed PMC passes
    (the newest of profiles/r06, r05, r04, r03 pmc_dominant.json; tools/pmc_dominant.sh + tools/pmc_summary.py):
    FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md "HBM") + WRITE_SIZE; None if it is for another
    kernel/shape."""
    for rnd in ("r06", "r05", "r04", "r03"):
        path = os.path.join(ROOT, "profiles", rnd, "pmc_dominant.json")
        if os.path.exists(path):
            break
    try:
        with open(path) as f:
            pm = json.load(f)
    except (OSError, ValueError):
        return {"traffic": None}
    if not kname.startswith(pm.get("kernel", "?")) or list(pm.get("shape_MNK", [])) != list(shape):
        return {"traffic": None}
    return {"traffic": pm["traffic_bytes"], "traffic_unit": "bytes/launch",
            "traffic_algorithmic": pm["algorithmic_bytes"], "traffic_source": os.path.relpath(path, ROOT)}


def cpu_baseline(seconds_budget=25.0):
    """The CPU restatement (oracle/pizero_oracle.py, fp32 torch-CPU) of the same bridge workload on this
    host's cores: fp32 fwd+bwd (the reported value), bf16-autocast fwd+bwd and one B=1 infer_action
    chunk (SURVEY 8(d) CPU-baseline legs).  Threads = the CPU-affinity count, capped by OMP_NUM_THREADS
    (the GPU box exports the job's CPU share there; its affinity mask lists the whole machine)."""
    from oracle import pizero_oracle as O

    affinity = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", affinity))
    threads = min(affinity, omp)
    torch.set_num_threads(threads)
    d = O.FULL_DIMS
    W = {}
    for k, shp in O.param_shapes(d).items():
        if ".mixtures.proprio." in k:
            continue
        W[k] = torch.empty(shp).uniform_(-0.02, 0.02).requires_grad_(k != "embed_tokens.weight")
    for k in list(W):
        if ".mixtures.action." in k:
            W[k.replace(".mixtures.action.", ".mixtures.proprio.")] = W[k]
    B = 1
    ids = torch.full((B, d["max_seq_len"]), d["image_token_index"], dtype=torch.int64)
    ids[:, 256] = 2
    ids[:, 257:275] = 1000
    ids[:, 275] = 108
    mask, vpos, ppos, apos = O.build_mask_and_positions(d, (ids != 0).long())
    pix = torch.rand(B, 3, 224, 224) * 2 - 1
    prop = torch.rand(B, 1, 7)
    act = torch.rand(B, 4, 7)
    t = torch.rand(B)
    x0 = torch.randn(B, 4, 7)

    def train_leg(n_max, budget, autocast):
        n, t0 = 0, time.perf_counter()
        while True:
            with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
                loss = O.pizero_loss(W, d, ids, pix, mask, vpos, ppos, apos, prop, act, t, x0)
            loss.backward()
            for v in W.values():
                v.grad = None
            n += 1
            el = time.perf_counter() - t0
            if el > budget or n >= n_max:
                return n * B / el, n, el

    fp32, n32, el32 = train_leg(3, 0.6 * seconds_budget, False)
    bf16, n16, el16 = train_leg(2, 0.25 * seconds_budget, True)
    itp, amask = O.split_mask(d, mask)
    with torch.no_grad():
        t0 = time.perf_counter()
        O.pizero_infer(W, d, ids, pix, itp, amask, vpos, ppos, apos, prop, torch.randn(B, 4, 7), clip=True)
        infer_ms = (time.perf_counter() - t0) * 1e3
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(line.split(":", 1)[1].strip() for line in f if line.startswith("model name"))
    except Exception:
        pass
    return {"value": fp32, "unit": "samples/s", "cores": threads, "kind": "port",
            "affinity_cpus": affinity, "omp_num_threads": omp, "cpu_model": cpu,
            "bf16_autocast_samples_s": bf16, "infer_action_ms_fp32_B1": infer_ms,
            "sample": (f"fp32: {n32} x bridge sample B=1 fwd+bwd in {el32:.1f}s; bf16-autocast: {n16} x in "
                       f"{el16:.1f}s; infer_action (prefill + 10 Euler steps, fp32, B=1) once; "
                       "torch-CPU oracle/pizero_oracle.py")}


def c5_inference(cfg, dev, iters):
    """BASELINE.json configs[4] (the Pi0-paper shape): 3 images (768 image tokens) + 20 text + 1 proprio,
    action chunk 50, B=1, bf16, prefill + 10 Euler steps in one hipGraph; against the 73 ms Pi0-paper
    figure quoted in the reference README (README.md:80,84).  Random-init weights."""
    import copy

    from pizero_native.graph import InferenceGraph
    from src.model.vla.pizero import PiZero

    c = copy.deepcopy(cfg)
    for key, val in (("num_images", 3), ("max_seq_len", 788), ("max_image_text_tokens", 788), ("horizon_steps", 50)):
        c[key] = val
    m = PiZero(c, device=dev, dtype=torch.bfloat16, init="default")
    m.tie_action_proprio_weights()
    m.freeze_all_weights()
    m.eval()
    d = m._engine().d
    gen = torch.Generator().manual_seed(11)
    ids = torch.full((1, d.P), 0, dtype=torch.int64)
    ids[:, : d.n_img] = d.image_token
    ids[:, d.n_img] = 2
    ids[:, d.n_img + 1 : d.P - 1] = torch.randint(3, 256000, (1, d.P - d.n_img - 2), generator=gen)
    ids[:, d.P - 1] = 108
    mask, vpos, ppos, apos = m.build_causal_mask_and_position_ids((ids != 0).long(), torch.bfloat16)
    itp, amask = m.split_full_mask_into_submasks(mask)
    pix = (torch.rand(1, 3, 3, d.img, d.img, generator=gen) * 2 - 1).to(dev, torch.bfloat16)
    prop = (torch.rand(1, 1, d.Pd, generator=gen) * 2 - 1).to(dev)
    noise = torch.randn(1, d.H, d.A, device=dev)
    def timed():
        g = InferenceGraph(m, 1)
        g.load(ids.to(dev), pix, m.block_prefix_counts(itp.to(dev), amask.to(dev)), vpos.to(dev), ppos.to(dev),
               apos.to(dev), prop, noise)
        g.capture()
        for _ in range(3):
            g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(iters):
            a = g.replay()
        e1.record()
        torch.cuda.synchronize()
        out = a.float().clone()
        # the two phases as separate graphs on the same static inputs (roofline of each): the prefill
        # (3 x SigLIP + the 789-row prefix pass writing the K/V cache) and the 10 denoise steps
        e, s = m._engine(), g.static
        pre_ms = _graph_ms(lambda: e.prefill(s["ids"], s["pix"], s["cnt"], s["vpos"], s["ppos"], s["proprios"],
                                              g.k, g.v), iters)

        def denoise():
            act = s["noise"].clone()
            t = torch.zeros(1, device=dev, dtype=torch.float32)
            for _ in range(d.steps):
                e.denoise_step(act, t, s["apos"], s["cnt"], g.k, g.v, 1)

        den_ms = _graph_ms(denoise, iters)
        return e0.elapsed_time(e1) / iters, out, pre_ms, den_ms

    ms, a16, pre16, den16 = timed()
    m.use_fp8_inference(True)  # BASELINE configs[4]: fp8 MFMA attention / MLP GEMMs
    ms8, a8, pre8, den8 = timed()
    rel = float((a8 - a16).norm() / a16.norm())
    # algorithmic budgets: prefill 3.711 TFLOP; denoise = 10 x every weight a denoise step reads
    # (the action expert's layers + final norm, the action encoder / decoder; its *proj.weight matrices e4m3 = 1 B
    # per element in fp8 mode, everything else bf16) + the K/V cache rows each step reads (bf16)
    sd = m.state_dict()
    den_keys = [k for k in sd if ".mixtures.action." in k or k.startswith(("action_encoder.", "action_decoder."))]
    n_proj = sum(sd[k].numel() for k in den_keys if ".mixtures.action." in k and k.endswith("proj.weight"))
    n_rest = sum(sd[k].numel() for k in den_keys) - n_proj
    kv = 10 * d.nL * (d.P + d.C + d.H) * d.hd * 2 * 2
    den_b16, den_b8 = 10 * (n_proj + n_rest) * 2 + kv, 10 * (n_proj * 1 + n_rest * 2) + kv

    def roof(pre, den, peak_tf, wbytes):
        return {"prefill": {"bound": "mfma", "ms": pre, "flop": C5_PREFILL_FLOP,
                            "achieved": C5_PREFILL_FLOP / (pre * 1e-3) / 1e12, "peak": peak_tf, "unit": "TFLOP/s",
                            "frac": C5_PREFILL_FLOP / (pre * 1e-3) / 1e12 / peak_tf},
                "denoise": {"bound": "hbm", "ms": den, "bytes": wbytes,
                            "achieved": wbytes / (den * 1e-3) / 1e9, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                            "frac": wbytes / (den * 1e-3) / 1e9 / PEAK_HBM_GBPS}}

    del m
    torch.cuda.empty_cache()
    return {"metric": "action-chunk infer ms, Pi0-paper shape (3 images = 768 img tokens + 20 text + "
                      "1 proprio, chunk 50, B=1, prefill + 10 Euler steps)",
            "graph_ms": ms, "dtype": "bf16", "fp8_graph_ms": ms8,
            "fp8": "e4m3 weights (per-tensor scales) for every SigLIP / vlm / action-expert Linear: prefill q|k|v and "
                   "MLP GEMMs W8A8 on the fp8 MFMA (per-row activation scales; the q|k|v / gate|up / fc1 inputs "
                   "quantised inside the preceding RMSNorm / LayerNorm), prefill o and the denoise W8A16 (codes expanded "
                   "to bf16); prefill joint attention QK^T and PV on the fp8 MFMA (pz_flash_fwd_f8: per-row Q / K, "
                   "per-head-dim V scales, P as e4m3(256 p)); SigLIP and denoise attention bf16",
            "fp8_vs_bf16_chunk_rel_l2": rel, "replays_timed": iters, "higher_is_better": False, "baseline_ms": 73.0,
            "baseline_source": "Pi0 paper figure quoted in the reference README.md:80,84 (other hardware)",
            "vs_baseline": 73.0 / ms, "fp8_vs_baseline": 73.0 / ms8,
            "roofline": {"bf16": roof(pre16, den16, PEAK_BF16_TFLOPS, den_b16),
                         "fp8": roof(pre8, den8, PEAK_FP8_TFLOPS, den_b8),
                         "note": "phases timed as separate hipGraphs on the graph's static inputs; prefill flop = the "
                                 "reference's FlopCounterMode count (SURVEY 8(d) C5), priced for fp8 against the fp8 "
                                 "dense peak although its o projection, SigLIP attention and few-row GEMMs run on the "
                                 "bf16 MFMA; denoise bytes = "
                                 "10 x (action-expert layers + norm + action encoder / decoder weights, proj weights "
                                 "1 B in fp8) + the K/V rows each step reads"}}


def _graph_ms(fn, iters):
    """ms per replay of fn captured into a hipGraph (two warm-up runs on a side stream first)"""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        fn()
    for _ in range(3):
        gr.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_envs(n, port, base=None):
    """The torchrun-style environment of each of n local ranks (reference: slurm/train_multi_gpu.sh:26-42 launches
    one process per GPU; scripts/run.py:39-47 reads LOCAL_RANK / WORLD_SIZE and sets the device from LOCAL_RANK)."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def visible_gpus():
    """GPUs this process may use, counted without touching HIP (a parent that initialised the GPU could not safely
    start its ranks): the GPU nodes of the KFD topology (simd_count > 0; CPU nodes have none), narrowed by
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES.  PZ_VISIBLE_GPUS overrides the count
    (CPU-host tests of the launcher only)."""
    if os.environ.get("PZ_VISIBLE_GPUS"):
        return int(os.environ["PZ_VISIBLE_GPUS"])
    base = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(base):
            try:
                with open(os.path.join(base, node, "properties")) as f:
                    props = dict(ln.split()[:2] for ln in f if len(ln.split()) >= 2)
            except OSError:
                continue
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except OSError:
        return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launch_ranks(n, argv):
    """``bench.py --gpus N`` started without a launcher: run N copies of this script, one per GPU, as children
    (before this process touches the GPU), inheriting stdout/stderr so rank 0's JSON line is the output.  A
    child that fails ends the others (they would wait in a collective); returns the worst exit code."""
    import signal
    import subprocess

    # PZ_RANKS_PER_GPU = k (one-card rehearsal, tests/test_bench_launcher.py): k ranks share each GPU, rank r on
    # device r // k -- applied in the children only; the parent's count is the same sysfs count as a real run's
    per = max(1, int(os.environ.get("PZ_RANKS_PER_GPU", "1")))
    have = visible_gpus()
    if have * per < n:
        print(f"bench.py: --gpus {n} but only {have} GPU(s) visible" + (f" ({per} ranks per GPU)" if per > 1 else ""),
              file=sys.stderr, flush=True)
        return 2

    def pdeathsig():  # a child outlives neither a killed parent nor its timeout
        import ctypes

        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG

    port = _free_port()
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=e, preexec_fn=pdeathsig)
             for e in rank_envs(n, port)]

    def stop_all(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + 20
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    signal.signal(signal.SIGTERM, lambda *a: (stop_all(), sys.exit(143)))
    worst = 0
    while any(p.poll() is None for p in procs):
        for p in procs:
            rc = p.poll()
            if rc not in (None, 0) and worst == 0:
                worst = rc if rc > 0 else 128 - rc
                print(f"bench.py: rank {procs.index(p)} exited with {rc}; stopping the other ranks", file=sys.stderr,
                      flush=True)
                stop_all()
        time.sleep(0.2)
    for p in procs:
        if p.returncode != 0 and worst == 0:
            worst = p.returncode if p.returncode > 0 else 128 - p.returncode
    return worst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU); without WORLD_SIZE in the environment bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--global-batch", type=int, default=1024)
    # 256 x 4 on one GPU: every per-micro-batch fixed cost (launch tails, norm / reduction passes, the loss, the
    # expert stream's join) paid 4 instead of 8 times and the 70656-row vlm GEMMs in whole 256-tile rounds --
    # measured 260.5 vs 252.5 samples/s for 128 x 8 on one box (profiles/r04/mb256_ab.txt; 247 GB peak of the
    # 288 GB), 128 x 8 255.7 vs 64 x 16 248.0 (profiles/r04/mb_ab.txt).  At 8 GPUs each rank runs 128 x 1.
    ap.add_argument("--micro-batch", type=int, default=256)
    ap.add_argument("--infer-iters", type=int, default=100)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-infer", action="store_true")
    ap.add_argument("--optim-bits", type=int, default=8, choices=(8, 32))
    ap.add_argument("--no-c5", action="store_true")
    ap.add_argument("--force-ddp", action="store_true",
                    help="run the data-parallel path (process group + PiZeroDDP bucketed RCCL all-reduce on the "
                         "comm stream) even at world size 1 (single-GPU check of the N>1 code path)")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus is not None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and args.gpus is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world} (launcher mismatch)", file=sys.stderr)
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # PZ_RANKS_PER_GPU / PZ_DIST_BACKEND: single-GPU rehearsal of the N>1 path (gloo, k ranks per card);
    # PZ_DEVICE: run a single process on another card
    per = max(1, int(os.environ.get("PZ_RANKS_PER_GPU", "1")))
    dev_idx = local // per if per > 1 else int(os.environ.get("PZ_DEVICE", local))
    backend = os.environ.get("PZ_DIST_BACKEND", "nccl")
    torch.cuda.set_device(dev_idx)
    dev = torch.device(f"cuda:{dev_idx}")
    ddp = world > 1 or args.force_ddp
    if ddp:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from pizero_native import ops
    from pizero_native.ddp import PiZeroDDP
    from pizero_native.graph import InferenceGraph
    from pizero_native.optim import FusedAdamW, clip_grad_norm_
    from src.model.vla.pizero import PiZero
    from src.utils.config import load_config

    cfg = load_config(os.path.join(ROOT, "open-pi-zero_amd", "config", "train", "bridge.yaml"))
    torch.manual_seed(1234 + rank)
    t0 = time.time()
    model = PiZero(cfg, use_ddp=world > 1, device=dev, dtype=torch.bfloat16, init="default")
    model.tie_action_proprio_weights()
    model.freeze_unused_weights()
    model.train()
    meta = PiZeroDDP(model, force_reduce=args.force_ddp) if ddp else model
    # the reference's optimizer is bnb AdamW8bit (train.py:171-175,194-198): blockwise 8-bit state
    opt_a = FusedAdamW(model.action_expert_parameters, lr=cfg.action_lr, weight_decay=cfg.action_weight_decay,
                       state_bits=args.optim_bits)
    opt_v = FusedAdamW(model.trainable_vlm_parameters, lr=cfg.vlm_lr, weight_decay=cfg.vlm_weight_decay,
                       state_bits=args.optim_bits)
    gb = args.global_batch
    mb = min(args.micro_batch, gb // world)
    accum = max(1, gb // (world * mb))
    gb = mb * accum * world
    gen = torch.Generator().manual_seed(rank)
    batches = [synthetic_batch(model, mb, dev, gen) for _ in range(min(accum, 2))]
    log(f"[bench] model ready in {time.time() - t0:.1f}s; world={world} micro_batch={mb} accum={accum} global={gb}")
    # per optimizer step (warm-up steps first): the sum of its micro-batch losses and the pre-clip gradient norm, kept
    # on the device (no host sync inside the timed region) and checked after it -- a non-finite loss or norm fails
    # the run (the reference logs the all-reduced loss of every micro-batch, train.py:399-410)
    n_all = args.warmup + args.steps
    step_loss = torch.zeros(n_all, device=dev)
    step_gnorm = torch.zeros(n_all, device=dev)

    def step(k):
        for i in range(accum):
            b = batches[i % len(batches)]
            last = i == accum - 1
            ctx = meta.no_sync() if (ddp and not last) else torch.enable_grad()
            with ctx:
                loss = meta(**b)
                (loss / accum).backward()
            step_loss[k:k + 1].add_(loss.detach())
        step_gnorm[k:k + 1].copy_(clip_grad_norm_([opt_a, opt_v], cfg.max_grad_norm))
        opt_a.step()
        opt_v.step()
        opt_a.zero_grad(set_to_none=True)
        opt_v.zero_grad(set_to_none=True)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize()
    if ddp:
        dist.barrier()
    # live probe of the dominant kernel: the vlm GeGLU gate|up GEMM (M = mb*276, N = 2*16384, K = 2048)
    d = model._engine().d
    Mg, Ng, Kg = mb * d.P, 2 * d.gI, d.gH
    probe = ops.set_probe(lambda M, N, K, epi, batch: (M, N, K, epi) == (Mg, Ng, Kg, ops.PZ_EPI_GEGLU))
    if ddp:
        meta.reducer.timing = True  # RCCL time per bucket + the un-hidden wait
        n_log0 = len(meta.reducer.log)
    torch.cuda.synchronize()
    if ddp:
        dist.barrier()
    t1 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    torch.cuda.synchronize()
    if ddp:
        dist.barrier()
    el = time.perf_counter() - t1
    ops.set_probe(None)
    elt = torch.tensor([el], device=dev)
    if ddp:
        dist.all_reduce(elt, op=dist.ReduceOp.MAX)
    el = float(elt.item())
    if ddp:  # every rank's micro-batch losses (outside the timed region)
        dist.all_reduce(step_loss)
    losses = [v / (accum * world) for v in step_loss.tolist()]  # mean micro-batch loss of each step
    gnorms = step_gnorm.tolist()
    if not all(math.isfinite(v) for v in losses + gnorms):  # no headline from a diverged run
        log(f"[bench] NON-FINITE training: loss per step {losses}, grad norm per step {gnorms} "
            f"({gb * args.steps / el:.1f} samples/s, not reported)")
        if ddp:
            dist.destroy_process_group()
        sys.exit(3)
    comm = None
    if ddp:
        # data parallelism keeps every replica's weights identical: a checksum of each rank's parameter arena
        # after the timed steps (outside the timed region)
        data = model._arena.data
        cs = torch.zeros(1, dtype=torch.float64, device=dev)
        for i in range(0, data.numel(), 1 << 26):
            cs += data[i:i + (1 << 26)].float().sum(dtype=torch.float64)
        css = [torch.zeros_like(cs) for _ in range(world)]
        dist.all_gather(css, cs)
        replicas_equal = all(torch.equal(c, css[0]) for c in css)
        if not replicas_equal:
            log(f"[bench] replica weight checksums differ: {[float(c) for c in css]}")
        meta.reducer.timing = False
        comm = meta.reducer.timing_summary(args.steps)
        if comm is not None:  # max over ranks (the slowest rank's communication sets the step)
            ct = torch.tensor([comm["comm_ms_per_step"], comm["exposed_ms_per_step"]], device=dev)
            dist.all_reduce(ct, op=dist.ReduceOp.MAX)
            comm["comm_ms_per_step"], comm["exposed_ms_per_step"] = float(ct[0]), float(ct[1])
            c, x = comm["comm_ms_per_step"], comm["exposed_ms_per_step"]
            comm["overlap_frac"] = 1.0 - x / c if c > 0 else None
            nbytes = sum(e for _, e in meta.reducer.log[n_log0:]) * model._arena.grad.element_size() / args.steps
            comm["bytes_per_step"] = nbytes
            comm["algbw_GBps"] = nbytes / (c * 1e-3) / 1e9 if c > 0 else None  # busbw = 2 (N-1) / N x algbw
    durs = [a.elapsed_time(b) for a, b in probe]
    kern_ms = sum(durs) / max(1, len(durs))
    flops_launch = 2.0 * Mg * Ng * Kg
    kname = ops.gemm_kernel_name(Mg, Ng, Kg, epi=ops.PZ_EPI_GEGLU, geglu_inter=d.gI)
    achieved = flops_launch / (kern_ms * 1e-3) / 1e12 if durs else None
    samples_s = gb * args.steps / el

    infer = None
    if not args.no_infer and rank == 0:
        batches = None
        torch.cuda.empty_cache()  # the training step's activation blocks (micro-batch 256: ~240 GB) go back
        model.eval()
        gi = synthetic_batch(model, 1, dev, torch.Generator().manual_seed(7))
        itp, amask = model.split_full_mask_into_submasks(gi["causal_mask"])
        noise = torch.randn(1, d.H, d.A, device=dev)
        # eager native path
        for _ in range(2):
            model.infer_action(gi["input_ids"], gi["pixel_values"], itp, amask, gi["vlm_position_ids"],
                               gi["proprio_position_ids"], gi["action_position_ids"], gi["proprios"], noise=noise)
        torch.cuda.synchronize()
        te = time.perf_counter()
        for _ in range(5):
            model.infer_action(gi["input_ids"], gi["pixel_values"], itp, amask, gi["vlm_position_ids"],
                               gi["proprio_position_ids"], gi["action_position_ids"], gi["proprios"], noise=noise)
        torch.cuda.synchronize()
        eager_ms = (time.perf_counter() - te) / 5 * 1e3
        g = InferenceGraph(model, 1)
        g.load(gi["input_ids"], gi["pixel_values"], model.block_prefix_counts(itp, amask), gi["vlm_position_ids"],
               gi["proprio_position_ids"], gi["action_position_ids"], gi["proprios"], noise)
        g.capture()
        for _ in range(3):
            g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(args.infer_iters):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        graph_ms = e0.elapsed_time(e1) / args.infer_iters
        # HBM roofline of the chunk: weights streamed once by the prefill (5.18 GB) + 10 x the
        # action expert (0.63 GB) + KV reads = 11.5 GB algorithmic bytes
        infer = {"metric": "bf16 action-chunk infer ms (B=1, prefill + 10 Euler steps)", "graph_ms": graph_ms,
                 "replays_timed": args.infer_iters, "eager_ms": eager_ms, "higher_is_better": False,
                 "baseline_ms": 75.0, "vs_baseline": 75.0 / graph_ms, "hbm_floor_ms": 1.44,
                 "algorithmic_bytes": INFER_BYTES, "achieved_GBps": INFER_BYTES / (graph_ms * 1e-3) / 1e9,
                 "frac": INFER_BYTES / (graph_ms * 1e-3) / (PEAK_HBM_GBPS * 1e9)}

    c5 = None
    if not args.no_infer and not args.no_c5 and rank == 0:
        c5 = c5_inference(cfg, dev, args.infer_iters)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline()

    if rank == 0:
        line = {
            "metric": "train samples/sec at gbsz 1024 (bf16 fwd+bwd+clip+AdamW)",
            "value": samples_s, "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random-init weights, random pixels/tokens/proprio/actions)",
            "config": {"workload": "Pi0 bridge training step: 256 img + 20 text + 1 proprio + 4 action tokens",
                       "model": "pi0 (SigLIP-So400m/14 + Gemma-2B + 0.3B action expert)", "global_batch": gb,
                       "micro_batch": mb, "grad_accum": accum, "seq_len": d.L,
                       "parallelism": f"dp{world}"},
            "ddp": None if not ddp else {
                "backend": dist.get_backend(), "buckets_reduced_per_step": sum(1 for _ in meta.reducer.log) / max(
                    1, args.steps + args.warmup), "async_rccl_buckets": sum(1 for a, _ in meta.reducer.log if a),
                "forced_at_world_1": bool(args.force_ddp and world == 1), "replica_weights_equal": replicas_equal,
                **(comm or {})},
            "mfma_frac_step": samples_s * TRAIN_FLOP_PER_SAMPLE / (world * PEAK_BF16_TFLOPS * 1e12),
            "roofline": {"bound": "mfma", "kernel": kname + " (vlm gate|up GeGLU GEMM)",
                         "shape_MNK": [Mg, Ng, Kg], "launches_timed": len(durs), "avg_launch_ms": kern_ms,
                         "achieved": achieved, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                         "frac": None if achieved is None else achieved / PEAK_BF16_TFLOPS,
                         **pmc_traffic(kname, [Mg, Ng, Kg])},
            "inference": infer,
            "c5_inference": c5,
            "cpu_baseline": cpu,
            "loss_mean": sum(losses[args.warmup:]) / args.steps,  # timed steps only
            "loss_per_step": losses, "grad_norm_per_step": gnorms,
            "peak_hbm_gb": torch.cuda.max_memory_allocated(dev) / 1e9 if dev.type == "cuda" else None,
            "optimizer": {"kind": f"AdamW, {args.optim_bits}-bit state" + (" (bnb AdamW8bit algorithm)" if
                                                                           args.optim_bits == 8 else ""),
                          "state_gb": (opt_a.state_bytes() + opt_v.state_bytes()) / 1e9},
        }
        print(json.dumps(line), flush=True)
    if ddp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

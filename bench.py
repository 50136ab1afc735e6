#!/usr/bin/env python3
"""Headline benchmark: images/s of DeiT-base/16-224 at bs=512 per GPU, bf16, on N MI355X GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W]             (N=1)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A step = one forward of the whole batch (patchify -> patch GEMM -> 12 x [LN, QKV GEMM,
attention, out-proj GEMM + residual, LN, FC1 GEMM + GELU, FC2 GEMM + residual] -> head) through
libevt_hip.so, plus, for N > 1, the RCCL all-gather of every rank's logits (the only exchange step
of the path: images are independent). Inputs are synthetic N(0,1) images already
resident in HBM; weights are the deterministic random init (no checkpoints exist offline).

Scaling modes (N > 1):
  weak (default)       each rank runs its own --batch images (512) per step: value = N*512/step;
  strong               --global-batch G: one global batch of G images, sharded over the ranks by
                       shard.sharded_forward (ceil/floor(G/N) per GPU), logits gathered by
                       shard.gather_logits; value = G/step (global 512 -> 64/GPU).
The process group has a timeout (--dist-timeout): a dead or hung peer ends the run with an error
instead of a hang (failure detection).

Extra objects on the JSON line:
  roofline      the dominant kernel (the role with the most device time; FC1 GEMM for DeiT-base,
                M = 512*197, K = 768, N = 3072) timed INSIDE 5 real forwards after the timed region:
                HIP events around each of its launches on the model's stream (evt_model_profile,
                edgevisiontransformer_amd/profiling.py; the same kernels the timed forwards run), so
                the figure agrees with the rocprofv3 kernel trace of the same command (its
                gemm_pers_kernel<35> launches); achieved = its algorithmic FLOPs (or bytes, for
                an HBM-bound role) / avg launch time vs the 2.5 PF dense bf16 MFMA peak (8 TB/s
                HBM); hbm_frac = algorithmic bytes / time / 8 TB/s for every role (per_role);
                traffic = HBM bytes per launch of the same role in real forwards of the same
                configuration, from the rocprofv3 PMC passes committed as
                profiles/pmc_<model>_<dtype>_bs<batch>.json (build commit reported beside it).
  cpu_baseline  the numpy fp32 restatement of the reference forward (oracle/, "port": TF is not
                installed anywhere), bs=1 forwards of the same model for ~15 s on the host BLAS
                threads.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_BF16_TFLOPS = 2516.6   # MI355X dense bf16 MFMA (spec; MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3     # MI355X fp32 matrix (spec)
PEAK_HBM_GBPS = 8000.0      # MI355X HBM3E (spec; MI355X_MICROARCH.md)
PMC_DIR = os.path.join(REPO, "profiles")  # pmc_<model>_<dtype>_bs<batch>.json (scripts/gpu_run.sh pmc:<name>:<role>:<args>)
def kernel_label(model: str, dtype: str, role: str) -> str:
    """The kernels a role's launches run (persistent 256x256 GEMM where the tile count fills the
    chip, else the 128x128 one; the fp32 path always the latter)."""
    swin = model.startswith("swin")
    gemm = "gemm_pers_kernel / gemm_nt_kernel" if dtype == "bf16" else "gemm_nt_kernel<float>"
    res = "BIAS|RESID|STATS" if swin else "BIAS|RESID|RESLN|STATS"
    names = {"fc1": f"{gemm}<LNIN|BIAS|{'GELU_ERF' if swin else 'GELU'}> (FC1)",
             "fc2": f"{gemm}<{res}> (FC2)", "out_proj": f"{gemm}<{res}> (out-proj)",
             "qkv": f"{gemm}<LNIN|BIAS> (QKV)",
             "attention": ("window_attn_bf16_kernel" if swin else
                           "attn_bf16_kernel" if dtype == "bf16" else "attn_f32_kernel"),
             "mlp": "swin_mlp96_kernel (stage-1 fused MLP)",
             "attn_sublayer": "swin_attn96_kernel (stage-1 fused attention sublayer)"}
    return names.get(role, role)
METRIC = "images/sec DeiT-base/16-224 bs=512 @1/2/4/8 GPU; % bf16 MFMA roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=512, help="images per GPU")
    ap.add_argument("--model", default="deit_base",
                    choices=["deit_base", "deit_small", "deit_tiny", "t2t_vit_7", "t2t_vit_10",
                             "t2t_vit_12", "t2t_vit_14", "swin_tiny", "swin_small", "swin_base"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline budget (0 = skip)")
    ap.add_argument("--no-probe", action="store_true", help="skip the per-kernel probe")
    ap.add_argument("--gemm-variant", type=int, default=0, help="evt_set_gemm_variant (tuning A/B)")
    ap.add_argument("--isolated-probe", action="store_true",
                    help="also time FC1 alone, back to back (reported as roofline.isolated_probe_us)")
    ap.add_argument("--probe-only", type=int, default=0, metavar="N",
                    help="only launch the FC1 probe kernel N times and exit (PMC collection)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: shard ONE global batch of this many images over the ranks")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="process-group (RCCL) timeout in seconds")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1: nccl (= RCCL over xGMI, one GPU per "
                         "rank) or gloo (host staging; ranks may share a GPU, so the N > 1 code "
                         "path runs on a one-GPU box: a plumbing check, not a scaling number)")
    ap.add_argument("--dump-logits", default="",
                    help="rank 0 writes the last step's gathered [global batch, classes] fp32 "
                         "logits to this .npy file (the multi-rank parity test)")
    return ap.parse_args()


def kernel_probe(dtype: str, M: int, K: int, N: int, iters: int = 20) -> float:
    """Average duration (s) of one FC1 GEMM launch exactly as the forward runs it (LayerNorm-
    folded input, bias, GELU epilogue: flags EPI_LNIN|EPI_BIAS|EPI_GELU), timed with HIP events
    on the stream the kernel is launched on."""
    from edgevisiontransformer_amd import _lib
    lib = _lib.load_library()
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float32
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev).manual_seed(123)
    x = torch.randn((M, K), generator=g, device=dev)
    A = x.to(tdt)
    stats = torch.zeros((M, 2 * ((K + 255) // 256), 2), device=dev)  # include/evt.h slot layout
    stats[:, 0, 0], stats[:, 0, 1] = x.sum(1), (x * x).sum(1)
    W = torch.randn((K, N), generator=g, device=dev) / K ** 0.5
    gam, bet = torch.ones(K, device=dev), torch.zeros(K, device=dev)
    kpad, npad = (K + 63) // 64 * 64, (N + 255) // 256 * 256
    wp = torch.empty((npad, kpad), dtype=tdt, device=dev)
    colsum, cvec = torch.empty(npad, device=dev), torch.empty(npad, device=dev)
    C = torch.empty((M, N), dtype=tdt, device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    _lib.check(lib.evt_pack_weight(_lib.DTYPE[dtype], P(W), P(gam), K, N, P(wp), kpad, npad, s))
    _lib.check(lib.evt_ln_fold(_lib.DTYPE[dtype], P(wp), kpad, npad, P(W), P(bet), None, K, N,
                               P(colsum), P(cvec), s))
    a = _lib.evt_dense_args()
    a.flags = _lib.EPI_LNIN | _lib.EPI_BIAS | _lib.EPI_GELU
    a.A, a.lda, a.Wp, a.Kpad, a.Npad = A.data_ptr(), K, wp.data_ptr(), kpad, npad
    a.C, a.ldc, a.M, a.N = C.data_ptr(), N, M, N
    a.bias, a.colsum, a.stats_in = cvec.data_ptr(), colsum.data_ptr(), stats.data_ptr()
    a.ln_width, a.ln_eps = K, 1e-5

    def launch():
        _lib.check(lib.evt_dense(_lib.DTYPE[dtype], ctypes.byref(a), s))
    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        launch()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / iters


def cpu_baseline(model_name: str, budget_s: float) -> dict:
    from edgevisiontransformer_amd.weights import make_images, make_t2t_params, make_vit_params
    if model_name.startswith("swin"):
        from oracle.swin_ref import swin_forward as fwd
        from edgevisiontransformer_amd.modeling.models.swin import swin_config_from_name
        from edgevisiontransformer_amd.weights import make_swin_params
        cfg = swin_config_from_name(f"{model_name}_patch4_window7_224")
        params = make_swin_params(cfg, seed=0)
        layout, src = "NCHW", "oracle/swin_ref.py"
    elif model_name.startswith("t2t"):
        from oracle.t2t_ref import t2t_vit_forward as fwd
        from edgevisiontransformer_amd.modeling.models.t2t_vit import t2t_cfg_for
        cfg = t2t_cfg_for(model_name)
        params = make_t2t_params(cfg, seed=0)
        layout, src = "NHWC", "oracle/t2t_ref.py"
    else:
        from oracle.vit_ref import vit_forward as fwd
        from edgevisiontransformer_amd.modeling.models.vit import _cfg_for as cfg_for
        cfg = cfg_for(model_name)
        params = make_vit_params(cfg, seed=0)
        layout, src = "NCHW", "oracle/vit_ref.py"
    vit_forward = fwd
    p32 = {k: v.astype(np.float32) for k, v in params.items()}
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:
        cores = os.cpu_count() or 1
    img = make_images(1, seed=99, layout=layout)
    vit_forward(p32, cfg, img, dtype=np.float32)  # warm BLAS
    n, t0 = 0, time.perf_counter()
    while True:
        vit_forward(p32, cfg, img, dtype=np.float32)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n >= 200:
            break
    return {"value": n / el, "unit": "images/s", "cores": int(cores), "kind": "port",
            "sample": f"{n} x {model_name} bs=1 forwards of the numpy fp32 restatement "
                      f"({src}) in {el:.1f} s; reference TF-CPU path not installable"}


def pmc_traffic(model: str, dtype: str, batch: int, role: str):
    """HBM bytes per launch of `role`'s kernels in real forwards of this configuration, from the
    rocprofv3 PMC passes committed as profiles/pmc_<model>_<dtype>_bs<batch>.json
    (scripts/gpu_run.sh pmc + scripts/pmc_roles.py: 2 x FETCH_SIZE, gfx950 tallies 128-B requests
    at 64 B, MI355X_MICROARCH.md HBM section, + WRITE_SIZE, averaged over the role's launches) and
    the build commit it measured. None if absent or collected for another role."""
    f = os.path.join(PMC_DIR, f"pmc_{model}_{dtype}_bs{batch}.json")
    try:
        d = json.load(open(f))
    except Exception:
        return None, None
    if d.get("batch") != batch:
        return None, None
    r = (d.get("roles") or {}).get(role) or (d if d.get("role") == role else None)
    if r is None:
        return None, None
    return r.get("traffic_bytes_per_launch"), {"file": os.path.relpath(f, REPO),
                                               "commit": d.get("commit"),
                                               "collected": d.get("collected")}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if local_rank >= ndev and not (world > 1 and args.dist_backend == "gloo"):
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local_rank} but {ndev} visible GPU(s) "
                         "(RCCL needs one GPU per rank; --dist-backend gloo may share them)")
    dev_index = local_rank % max(ndev, 1)
    torch.cuda.set_device(dev_index)
    dist = None
    gloo = world > 1 and args.dist_backend == "gloo"
    if world > 1:
        import datetime
        import torch.distributed as dist
        if gloo:
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=args.dist_timeout))
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index),
                                    timeout=datetime.timedelta(seconds=args.dist_timeout))

    if args.probe_only:
        from edgevisiontransformer_amd.modeling.models.vit import _cfg_for
        cfg = _cfg_for(args.model)
        t = kernel_probe(args.dtype, args.batch * cfg.tokens, cfg.dim, cfg.ffn[0], iters=args.probe_only)
        print(json.dumps({"probe_us": round(t * 1e6, 1), "M": args.batch * cfg.tokens, "K": cfg.dim,
                          "N": cfg.ffn[0]}), flush=True)
        return
    from edgevisiontransformer_amd import shard
    t2t = args.model.startswith("t2t")
    swin = args.model.startswith("swin")
    if swin:
        from edgevisiontransformer_amd.modeling.models import swin as mod
    elif t2t:
        from edgevisiontransformer_amd.modeling.models import t2t_vit as mod
    else:
        from edgevisiontransformer_amd.modeling.models import vit as mod
    strong = args.global_batch > 0
    if strong:  # this rank's shard of one global batch (shard.shard_range)
        s0, s1 = shard.shard_range(args.global_batch, world, rank)
        B, G = s1 - s0, args.global_batch
        cap = -(-G // world)
    else:
        B, G, cap = args.batch, world * args.batch, args.batch
    model = mod.build_named(args.model, dtype=args.dtype, seed=0, max_batch=cap)
    if args.gemm_variant:
        from edgevisiontransformer_amd import _lib
        _lib.check(_lib.load_library().evt_set_gemm_variant(args.gemm_variant))
    shape = (224, 224, 3) if t2t else (3, 224, 224)   # T2T-ViT is channel-last
    if strong:  # every rank holds the global batch (same seed): sharded_forward slices its shard
        g = torch.Generator(device="cuda").manual_seed(1000)
        gimg = torch.randn((G, *shape), generator=g, device="cuda", dtype=torch.float32)
        img = gimg[s0:s1]
    else:
        g = torch.Generator(device="cuda").manual_seed(1000 + rank)
        img = torch.randn((B, *shape), generator=g, device="cuda", dtype=torch.float32)
    logits = torch.empty((max(B, 1), model.num_classes), device="cuda", dtype=torch.float32)
    gathered = None
    if world > 1 and not strong:  # gloo moves host tensors (shard.gather_logits stages the same way)
        gathered = torch.empty((world * B, model.num_classes), device="cpu" if gloo else "cuda")
    last = {}

    def local_forward(x):
        return model.forward_into(x, logits[: x.shape[0]])

    def step():
        if strong:
            last["logits"] = shard.sharded_forward(local_forward, gimg, world, rank)
        else:
            model.forward_into(img, logits)
            if world > 1:
                dist.all_gather_into_tensor(gathered, logits.cpu() if gloo else logits)
            last["logits"] = gathered if world > 1 else logits

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device="cpu" if gloo else "cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ok = bool(torch.isfinite(logits[:B]).all().item())
    if args.dump_logits and rank == 0:
        np.save(args.dump_logits, last["logits"].float().cpu().numpy())

    gflop_img = model.cfg.gflop_per_image()
    imgs_per_s = G * args.steps / el
    peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
    roof = None
    if rank == 0 and not args.no_probe:
        # every role's kernels timed INSIDE real forwards (HIP events around each launch on the
        # model's stream, evt_model_profile) with their algorithmic work, after the timed region
        from edgevisiontransformer_amd.profiling import kernel_times, roofline_table
        kt = kernel_times(model, img, logits[:B], forwards=5)
        table = roofline_table(kt, peak, PEAK_HBM_GBPS)
        dom = max(kt, key=lambda r: kt[r]["us_per_forward"])
        k = kt[dom]
        t_k = k["us_per_launch"] * 1e-6
        fl, by = k["gflop"] * 1e9 / k["launches"], k["gbytes"] * 1e9 / k["launches"]
        mfma_bound = fl / peak / 1e12 >= by / PEAK_HBM_GBPS / 1e9
        ach = fl / t_k / 1e12 if mfma_bound else by / t_k / 1e9
        roof = {"bound": "mfma" if mfma_bound else "hbm", "achieved": round(ach, 2),
                "peak": peak if mfma_bound else PEAK_HBM_GBPS,
                "unit": "TFLOP/s" if mfma_bound else "GB/s",
                "frac": round(ach / (peak if mfma_bound else PEAK_HBM_GBPS), 4),
                "traffic": None, "role": dom,
                "kernel": f"{kernel_label(args.model, args.dtype, dom)} ({args.model}, {args.dtype})",
                "algorithmic_flop_per_launch": fl, "algorithmic_bytes_per_launch": by,
                "hbm_gbps": round(by / t_k / 1e9, 1),
                "hbm_frac": round(by / t_k / 1e9 / PEAK_HBM_GBPS, 4),
                "mfma_frac": round(fl / t_k / 1e12 / peak, 4),
                "avg_launch_us": round(t_k * 1e6, 1), "launches_timed": 5 * k["launches"],
                "timing": "HIP events around each launch of the role inside 5 forwards "
                          "(evt_model_profile) of the kernels the timed forwards run",
                "per_role": table}
        roof["traffic"], roof["traffic_source"] = pmc_traffic(args.model, args.dtype, cap, dom)
        if dom == "fc1" and not t2t and not swin:
            M, K, N = B * model.cfg.tokens, model.cfg.dim, model.cfg.ffn[0]
            roof["kernel"] += f" M={M} K={K} N={N}"
            if args.isolated_probe:  # off by default: its launches would mix into a rocprof average
                roof["isolated_probe_us"] = round(kernel_probe(args.dtype, M, K, N) * 1e6, 1)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(args.model, args.cpu_seconds)
    if rank == 0:
        coll = "gloo all-gather of logits, ranks sharing GPUs" if gloo else "RCCL all-gather of logits"
        par = "dp1" if world == 1 else (
            f"dp{world} (one global batch of {G} sharded {B}-{cap} per GPU, {coll})"
            if strong else f"dp{world} (batch shard, {coll})")
        out = {
            "metric": METRIC if args.model == "deit_base" else f"images/sec {args.model} bs={B}",
            "value": round(imgs_per_s, 2), "unit": "images/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic N(0,1) images resident in HBM; deterministic random-init weights",
            "config": {"workload": f"{args.model}/{'224' if t2t or swin else '16-224'} forward, "
                                   f"bs={cap} per GPU, {args.dtype}",
                       "model": args.model, "global_batch": G, "per_gpu_batch": cap,
                       "seq_len": model.cfg.res(0) ** 2 if swin else model.cfg.tokens,
                       "parallelism": par,
                       "gemm_variant": args.gemm_variant or "automatic",
                       # batch lanes of the handle (evt_model_set_lanes); the roofline's per-role
                       # times come from profiled forwards, which run as one lane
                       "lanes": model.lanes()},
            "model_roofline": {"achieved_tflops": round(imgs_per_s * gflop_img / world / 1e3, 2),
                               "peak": peak, "frac": round(imgs_per_s * gflop_img / world / 1e3
                                                           / peak, 4),
                               "gflop_per_image": round(gflop_img, 3)},
            "roofline": roof, "cpu_baseline": cpu, "logits_finite": ok,
        }
        if world > 1:
            out["dist_backend"] = args.dist_backend
            out["devices"] = ndev
            if gloo:
                out["note"] = ("gloo plumbing run of the N > 1 code path (ranks may share a GPU): "
                               "not a scaling measurement")
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Benchmark CLI of the MI355X ViT path, mirroring the reference `tools.py` conventions.

    python -m edgevisiontransformer_amd.tools gpu_benchmark --model deit_base --input_shape 512,3,224,224
    python -m edgevisiontransformer_amd.tools gpu_benchmark --model deit_tiny --prune_encoding all_head2_ffn0.7
    python -m edgevisiontransformer_amd.tools test_keras_latency --model t2t_vit_14 --input_shape 1,224,224,3
    python -m edgevisiontransformer_amd.tools prune_benchmark --types tiny --num_runs 20
    python -m edgevisiontransformer_amd.tools fetch_latency_std -f bench.log

Reference conventions kept (so existing `run.sh`-style sweeps and log scrapers work unchanged):
  * `sys.argv[1]` selects the sub-command (reference tools.py:1011-1086);
  * `gpu_benchmark` takes the `server_benchmark` flag set (tools.py:7-67): --model, --num_runs (50),
    --warmup_runs (50), --top (average of the K shortest), --precision (2..6), --input_shape
    (comma list), --io_binding, and accepts --use_gpu / --intra_op_threads / --dtype float32 as
    no-ops; latency is `timeit.default_timer` around one call, host-synchronised, and the line is
    printed exactly as tools.py:116 does: "{name}  Avg latency: {ms} ms, Std: {ms} ms.";
  * `test_keras_latency` (tools.py:170-213): --test_times + 1 calls, the first dropped,
    "Avg latency: {ms}ms";
  * `prune_benchmark` builds the ViT_Pruned sweep of experiments.py:150-204 (PruneBenchmark);
  * `fetch_latency_std` parses such logs like utils.py:409-462.
Without --io_binding the input is a host numpy batch (the call includes the host->device copy
and the logits copy back, as ONNX Runtime's session.run does); with --io_binding the batch and
logits stay resident in HBM.
"""
from __future__ import annotations

import argparse
import os
import sys
import timeit
from typing import List, Optional

import numpy as np

VIT_NAMED = {"deit_tiny": 3, "deit_small": 6, "deit_base": 12}   # heads (vit.py:100-109)
T2T_NAMED = ("t2t_vit_7", "t2t_vit_10", "t2t_vit_12", "t2t_vit_14")
SWIN_NAMED = ("swin_tiny", "swin_small", "swin_base")   # get_swin configs (tools.py:282)


def build_model(name: str, compute_dtype: str, prune_encoding: Optional[str] = None,
                max_batch: int = 1, seed: int = 0):
    """A model by reference name (deit_*, t2t_vit_*, swin_*), optionally head/FFN pruned."""
    if name in SWIN_NAMED or name.startswith("swin_") and name.endswith("_224"):
        if prune_encoding:
            raise ValueError("prune_encoding applies to DeiT models only")
        from .modeling.models.swin import get_swin
        cfg_name = name if name.endswith("_224") else f"{name}_patch4_window7_224"
        return get_swin(cfg_name, dtype=compute_dtype, seed=seed, max_batch=max_batch)
    if name in T2T_NAMED:
        if prune_encoding:
            raise ValueError("prune_encoding applies to DeiT models only")
        from .modeling.models.t2t_vit import build_named
        return build_named(name, dtype=compute_dtype, seed=seed, max_batch=max_batch)
    if name not in VIT_NAMED:
        raise ValueError(f"unknown model {name!r}; one of "
                         f"{sorted(VIT_NAMED) + list(T2T_NAMED) + list(SWIN_NAMED)}")
    from .modeling.models.vit import ViT_Pruned, build_named
    if prune_encoding:
        h = VIT_NAMED[name]
        return ViT_Pruned(dim=h * 64, depth=12, heads=h, mlp_dim=h * 64 * 4, head_size=64,
                          prune_encoding=prune_encoding, dtype=compute_dtype, seed=seed,
                          max_batch=max_batch)
    return build_named(name, dtype=compute_dtype, seed=seed, max_batch=max_batch)


def _input_shape(name: str, spec: Optional[str]) -> List[int]:
    if spec:
        return [int(x) for x in spec.split(",")]
    return [1, 224, 224, 3] if name in T2T_NAMED else [1, 3, 224, 224]


def latency_samples(model, shape: List[int], num_runs: int, warmup_runs: int,
                    io_binding: bool, seed: int = 0, graph: bool = False) -> List[float]:
    """Seconds per call, `timeit.default_timer` around one host-synchronised forward
    (graph: replay of a captured HIP graph of the device-resident forward)."""
    import torch
    rng = np.random.default_rng(seed)
    host = rng.standard_normal(shape, dtype=np.float32)   # tools.py:204 / utils.py:482 style
    dev = torch.from_numpy(host).to(model.device)
    logits = torch.empty((shape[0], model.num_classes), dtype=torch.float32, device=model.device)

    if graph:
        model.capture_graph(dev, logits)

    def run():
        if graph:
            model.replay_graph()
            torch.cuda.synchronize(model.device)
        elif io_binding:
            model.forward_into(dev, logits)
            torch.cuda.synchronize(model.device)
        else:
            model(host)  # numpy in -> numpy out (includes both copies)

    for _ in range(warmup_runs):
        run()
    out = []
    for _ in range(num_runs):
        t0 = timeit.default_timer()
        run()
        out.append(timeit.default_timer() - t0)
    return out


def summarize(latencies: List[float], top: Optional[int]) -> tuple:
    lat = sorted(latencies)
    if top:
        lat = lat[:top]
    return float(np.average(lat)), float(np.std(lat))


def format_line(name: str, avg_s: float, std_s: float, precision: int) -> str:
    """tools.py:116 format (two spaces after the name, a space inside each number field)."""
    return (f"{name}  Avg latency: {avg_s * 1000: .{precision}f} ms, "
            f"Std: {std_s * 1000: .{precision}f} ms.")


def _server_flags(parser: argparse.ArgumentParser) -> None:
    parser.add_argument("func", help="specify the work to do.")
    parser.add_argument("--model", required=True, type=str,
                        help=f"model name: {', '.join(list(VIT_NAMED) + list(T2T_NAMED))}")
    parser.add_argument("--prune_encoding", default=None, type=str,
                        help="ViT_Pruned encoding (all_head{N}_ffn{F} / layerwise_h{N}-d{F}_...)")
    parser.add_argument("--use_gpu", action="store_true", help="accepted; always the GPU")
    parser.add_argument("--num_runs", type=int, default=50)
    parser.add_argument("--warmup_runs", type=int, default=50)
    parser.add_argument("--dtype", default="float32", type=str, help="input data type (float32)")
    parser.add_argument("--compute_dtype", default="bf16", choices=["bf16", "f32", "mx8"],
                        help="mx8: MXFP8 encoder Dense layers (ViT family; the quantization axis)")
    parser.add_argument("--intra_op_threads", type=int, default=1, help="accepted; unused")
    parser.add_argument("--top", type=int, default=None,
                        help="number of shortest runs to take average")
    parser.add_argument("--io_binding", action="store_true", dest="io_binding")
    parser.add_argument("--graph", action="store_true",
                        help="replay a captured HIP graph of the device-resident forward")
    parser.add_argument("--precision", default=2, choices=[2, 3, 4, 5, 6], type=int)
    parser.add_argument("--input_shape", default=None, type=str, help="input_shape")


def gpu_benchmark(argv: Optional[List[str]] = None) -> str:
    parser = argparse.ArgumentParser()
    _server_flags(parser)
    args = parser.parse_args(argv)
    if args.dtype != "float32":
        raise ValueError("input dtype must be float32 (the reference forward's input)")
    shape = _input_shape(args.model, args.input_shape)
    model = build_model(args.model, args.compute_dtype, args.prune_encoding, max_batch=shape[0])
    lat = latency_samples(model, shape, args.num_runs, args.warmup_runs, args.io_binding,
                          graph=args.graph)
    avg, std = summarize(lat, args.top)
    name = args.model + (f"_{args.prune_encoding}" if args.prune_encoding else "")
    line = format_line(name, avg, std, args.precision)
    print(line, flush=True)
    return line


def test_keras_latency(argv: Optional[List[str]] = None) -> str:
    parser = argparse.ArgumentParser()
    parser.add_argument("func")
    parser.add_argument("--model", required=True, type=str)
    parser.add_argument("--use_gpu", action="store_true")
    parser.add_argument("--test_times", type=int, default=5)
    parser.add_argument("--input_shape", required=True, type=str)
    parser.add_argument("--compute_dtype", default="bf16", choices=["bf16", "f32", "mx8"],
                        help="mx8: MXFP8 encoder Dense layers (ViT family; the quantization axis)")
    args = parser.parse_args(argv)
    shape = _input_shape(args.model, args.input_shape)
    model = build_model(args.model, args.compute_dtype, max_batch=shape[0])
    print(f"Successfully loaded model from {args.model}.")
    lat = latency_samples(model, shape, args.test_times + 1, 0, io_binding=False)
    line = f"Avg latency: {np.average(lat[1:]) * 1000: .2f}ms"
    print(line, flush=True)
    return line


def prune_encodings(types=("tiny", "small", "base")) -> List[tuple]:
    """(model, encoding) pairs of the reference PruneBenchmark (experiments.py:150-204)."""
    heads = {"tiny": 3, "small": 6, "base": 12}
    out = []
    for t in types:
        for thr in range(10, 100, 10):                       # _add_ffn_only_models
            out.append((f"deit_{t}", f"all_head{heads[t]}_ffn{thr / 100}"))
    for t in types:
        for h in range(1, heads[t]):                         # _add_head_only_models
            out.append((f"deit_{t}", f"all_head{h}_ffn1.0"))
    extra = {"tiny": [f"all_head2_ffn{x}" for x in (0.7, 0.8, 0.9)],
             "small": [f"all_head{i}_ffn{j}" for i in (4, 5) for j in (0.6, 0.7, 0.8, 0.9)]}
    for t in types:                                          # _add_head_ffn_models
        out += [(f"deit_{t}", e) for e in extra.get(t, [])]
    return out


def prune_benchmark(argv: Optional[List[str]] = None) -> List[str]:
    parser = argparse.ArgumentParser()
    parser.add_argument("func")
    parser.add_argument("--types", default="tiny,small,base", type=str)
    parser.add_argument("--batch", type=int, default=1, help="reference models are b1")
    parser.add_argument("--num_runs", type=int, default=50)
    parser.add_argument("--warmup_runs", type=int, default=10)
    parser.add_argument("--top", type=int, default=None)
    parser.add_argument("--precision", default=2, choices=[2, 3, 4, 5, 6], type=int)
    parser.add_argument("--compute_dtype", default="bf16", choices=["bf16", "f32", "mx8"],
                        help="mx8: MXFP8 encoder Dense layers (ViT family; the quantization axis)")
    parser.add_argument("--io_binding", action="store_true")
    args = parser.parse_args(argv)
    lines = []
    for model_name, enc in prune_encodings(tuple(args.types.split(","))):
        m = build_model(model_name, args.compute_dtype, enc, max_batch=args.batch)
        lat = latency_samples(m, [args.batch, 3, 224, 224], args.num_runs, args.warmup_runs,
                              args.io_binding)
        avg, std = summarize(lat, args.top)
        line = format_line(f"{model_name}_b{args.batch}_{enc}", avg, std, args.precision)
        print(line, flush=True)
        lines.append(line)
        m.close()
    return lines


def _fetch_float(text: str, marker: str) -> Optional[float]:
    """utils.py:409-427: the number following `marker` in `text`, or None."""
    begin = text.find(marker)
    if begin == -1:
        return None
    begin += len(marker)
    while begin < len(text) and not text[begin].isnumeric():
        begin += 1
    end = begin
    while end < len(text) and (text[end].isnumeric() or text[end] == "."):
        end += 1
    return float(text[begin:end]) if end > begin else None


def fetch_latency_std(argv: Optional[List[str]] = None) -> dict:
    """utils.py:429-462 over our log lines ("{name}  Avg latency: ..."): names are the text
    before "  Avg latency" (the reference takes .tflite file-name lines)."""
    parser = argparse.ArgumentParser()
    parser.add_argument("func")
    parser.add_argument("--file", "-f", required=True, type=str)
    parser.add_argument("--begin_line", default=0, type=int)
    parser.add_argument("--end_line", default=None, type=int)
    parser.add_argument("--precision", default=2, type=int)
    args = parser.parse_args(argv)
    with open(args.file) as f:
        lines = f.readlines()[args.begin_line:args.end_line]
    names, lat, std = [], [], []
    for line in lines:
        raw = line.rstrip("\n")
        low = raw.lower()
        if "  avg latency" in low:
            names.append(raw[:low.index("  avg latency")])
        v = _fetch_float(low, "latency")
        if v is not None:
            lat.append(v)
        s = _fetch_float(low, "std")
        if s is not None:
            std.append(s)
    print("name", *names)
    print("latency", [round(x, args.precision) for x in lat])
    print("std", [round(x, args.precision) for x in std])
    return {"name": names, "latency": lat, "std": std}


COMMANDS = {
    "gpu_benchmark": gpu_benchmark,
    "server_benchmark": gpu_benchmark,   # the reference name of the same flag set
    "test_keras_latency": test_keras_latency,
    "prune_benchmark": prune_benchmark,
    "fetch_latency_std": fetch_latency_std,
}


def main(argv: Optional[List[str]] = None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in COMMANDS:
        print(f"usage: python -m edgevisiontransformer_amd.tools {{{','.join(COMMANDS)}}} ...",
              file=sys.stderr)
        sys.exit(2)
    COMMANDS[argv[0]](argv)


if __name__ == "__main__":
    main()

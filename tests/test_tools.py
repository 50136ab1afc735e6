"""The tools.py-compatible CLI (edgevisiontransformer_amd/tools.py): output format, log parsing
and the prune sweep on the host; a short GPU run of each sub-command."""
import numpy as np
import pytest

from edgevisiontransformer_amd import tools


def test_format_matches_reference_line():
    # reference tools.py:116: f'{name}  Avg latency: {avg*1000: .{p}f} ms, Std: {std*1000: .{p}f} ms.'
    avg, std, p = 0.0123456, 0.000789, 3
    ref = f"deit_tiny  Avg latency: {avg * 1000: .{p}f} ms, Std: {std * 1000: .{p}f} ms."
    assert tools.format_line("deit_tiny", avg, std, p) == ref


def test_summarize_top_k_shortest():
    avg, std = tools.summarize([5.0, 1.0, 3.0, 2.0], top=2)
    assert avg == 1.5 and std == pytest.approx(0.5)


def test_fetch_latency_std_roundtrip(tmp_path, capsys):
    log = tmp_path / "bench.log"
    log.write_text(tools.format_line("deit_base", 0.0105, 0.0002, 2) + "\n" +
                   tools.format_line("t2t_vit_14", 0.0071, 0.0001, 2) + "\n")
    out = tools.fetch_latency_std(["fetch_latency_std", "-f", str(log)])
    assert out["name"] == ["deit_base", "t2t_vit_14"]
    assert out["latency"] == [10.5, 7.1] and out["std"] == [0.2, 0.1]


def test_prune_sweep_matches_reference_prunebenchmark():
    """experiments.py:150-204: 9 FFN-only + (H-1) head-only per size, plus the head+FFN extras."""
    pairs = tools.prune_encodings()
    assert len(pairs) == (9 + 2 + 3) + (9 + 5 + 8) + (9 + 11)
    assert ("deit_tiny", "all_head2_ffn0.7") in pairs and ("deit_base", "all_head12_ffn0.1") in pairs
    from edgevisiontransformer_amd.modeling.models.vit import decode_prune_encoding
    for _, enc in pairs:
        decode_prune_encoding(enc)


@pytest.mark.gpu
def test_gpu_benchmark_runs(gpu, capsys):
    line = tools.gpu_benchmark(["gpu_benchmark", "--model", "deit_tiny", "--num_runs", "3",
                                "--warmup_runs", "1", "--input_shape", "2,3,224,224", "--top", "2"])
    assert line.startswith("deit_tiny  Avg latency: ") and line.endswith(" ms.")
    line = tools.gpu_benchmark(["gpu_benchmark", "--model", "deit_tiny", "--prune_encoding",
                                "all_head2_ffn0.7", "--num_runs", "2", "--warmup_runs", "1",
                                "--io_binding", "--precision", "4"])
    assert line.startswith("deit_tiny_all_head2_ffn0.7  Avg latency: ")
    line = tools.gpu_benchmark(["gpu_benchmark", "--model", "t2t_vit_7", "--num_runs", "3",
                                "--warmup_runs", "1", "--graph"])
    assert line.startswith("t2t_vit_7  Avg latency: ")
    line = tools.test_keras_latency(["test_keras_latency", "--model", "t2t_vit_7", "--test_times",
                                     "2", "--input_shape", "1,224,224,3"])
    assert line.startswith("Avg latency: ") and line.endswith("ms")

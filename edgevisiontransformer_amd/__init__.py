"""edgevisiontransformer_amd - MI355X-native (gfx950) inference path for the vision transformers of
xudoong/EdgeVisionTransformer's `modeling.models` (DeiT / ViT / ViT_Pruned, T2T-ViT) and the Swin
Transformer its `tools.py` benchmarks through `get_swin`.

Host code is Python on PyTorch-ROCm calling libevt_hip.so (C ABI: include/evt.h), whose hot
kernels (patchify / unfold, MFMA GEMMs with fused LayerNorm / GELU / residual epilogues, fused and
windowed attention, the TokenPerformer) are hand-written HIP for CDNA4. Import of the model
classes is lazy so that host-only utilities (weights, prune encodings, CLI parsing) work without a
GPU.
"""
__version__ = "0.4.0"

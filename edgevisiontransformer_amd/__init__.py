"""edgevisiontransformer_amd - MI355X-native (gfx950) inference path for the ViT family of
xudoong/EdgeVisionTransformer's `modeling.models` (DeiT / ViT_Pruned; T2T-ViT next).

Host code is Python on PyTorch-ROCm calling libevt_hip.so (C ABI: include/evt.h), whose hot
kernels (patchify, MFMA GEMM with fused epilogues, fused attention, LayerNorm) are hand-written
HIP for CDNA4. Import of the model classes is lazy so that host-only utilities (weights, prune
encodings, CLI parsing) work without a GPU.
"""
__version__ = "0.1.0"

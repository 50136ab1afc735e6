"""Mirror of the reference `modeling.models`: vit.py (ViT, ViT_Pruned, get_deit_*), t2t_vit.py
(T2T_ViT, get_t2t_vit_*) and the Swin Transformer of utils.py:get_swin."""

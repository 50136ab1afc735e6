"""Mirror of the reference `modeling.models` (vit.py; t2t_vit.py next)."""

"""Mirror of the reference `modeling` package for the ViT inference path."""

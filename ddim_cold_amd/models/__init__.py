"""Model families: the ViT diffusion denoiser (`DiffusionVisionTransformer`)."""
from .vit import (Attention, Block, DiffusionVisionTransformer, DropPath, Mlp, PatchEmbed, drop_path,
                  positionalencoding1d, sinusoidal_timestep_embedding, trunc_normal_)
from .configs import MODEL_CONFIGS, build_model

__all__ = ["Attention", "Block", "DiffusionVisionTransformer", "DropPath", "Mlp", "PatchEmbed", "drop_path",
           "positionalencoding1d", "sinusoidal_timestep_embedding", "trunc_normal_", "MODEL_CONFIGS",
           "build_model"]

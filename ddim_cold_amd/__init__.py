"""ddim_cold_amd — an MI355X-native (gfx950 / CDNA4) DDIM & cold-diffusion ViT framework.

Capabilities of nyyxxx/DDIM-COLD (DiffusionVisionTransformer API, YAML
experiment schema, multi_gpu_trainer entry point, .pkl checkpoint layout,
DDIM / cold / img2img samplers) re-designed around hand-written HIP kernels,
hipGraph-captured steps and RCCL data parallelism.
"""
__version__ = "0.1.0"

from .models import DiffusionVisionTransformer, build_model, MODEL_CONFIGS  # noqa: E402

__all__ = ["DiffusionVisionTransformer", "build_model", "MODEL_CONFIGS", "__version__"]

"""zipvoice_amd — MI355X-native ZipVoice inference engine (hot path: flow-matching
decoder + Euler ODE loop as hand-written HIP kernels for gfx950)."""
from .config import ModelConfig, default_config  # noqa: F401

"""Flow-matching Euler solver — same interface as the reference's
``zipvoice/models/modules/solver.py`` (EulerSolver :168-240, DistillEulerSolver
:243-253, get_time_steps :256-281), with the whole N-step loop (CFG batch
doubling, guidance combine and the Euler update) running inside the HIP engine
(``zv_euler_sample``): no host synchronisation between steps."""
from __future__ import annotations

from typing import Union

import torch


def get_time_steps(t_start: float = 0.0, t_end: float = 1.0, num_step: int = 10,
                   t_shift: float = 1.0, device=torch.device("cpu")) -> torch.Tensor:
    """solver.py:256-281 (the engine computes the same grid internally)."""
    ts = torch.linspace(t_start, t_end, num_step + 1).to(device)
    return t_shift * ts / (1 + (t_shift - 1) * ts)


class EulerSolver:
    def __init__(self, model, func_name: str = "forward_fm_decoder"):
        self.model = model
        self.func_name = func_name

    def sample(self, x: torch.Tensor, text_condition: torch.Tensor,
               speech_condition: torch.Tensor, padding_mask: torch.Tensor, num_step: int = 10,
               guidance_scale: Union[float, torch.Tensor] = 0.0, t_start: float = 0.0,
               t_end: float = 1.0, t_shift: float = 1.0, **kwargs) -> torch.Tensor:
        """guidance_scale: a float or a tensor of shape (batch, 1, 1) (solver.py:61-62):
        per-utterance scales run the same CFG loop with g per row."""
        assert isinstance(t_start, float) and isinstance(t_end, float)
        if torch.is_tensor(guidance_scale) and guidance_scale.numel() == 1:
            guidance_scale = float(guidance_scale)
        if not torch.is_tensor(guidance_scale):
            guidance_scale = float(guidance_scale)
        return self.model.engine.euler_sample(x, text_condition, speech_condition, padding_mask,
                                              num_step, guidance_scale, t_start, t_end, t_shift)


class DistillEulerSolver(EulerSolver):
    """Same loop; the engine knows the model is distilled (no CFG doubling, the
    guidance scale goes through the guidance embedding, solver.py:127-165)."""

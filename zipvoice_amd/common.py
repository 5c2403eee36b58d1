"""Host-side integer helpers of the inference path (token padding, masks,
frame->token durations).  Mirrors ``zipvoice/utils/common.py`` of the
reference: these run on the host in the reference too (python loops), and
touch only token ids and lengths."""
from __future__ import annotations

from typing import List

import torch


def pad_labels(y: List[List[int]], pad_id: int, device=None) -> torch.Tensor:
    """common.py:255-268: append ONE pad to every row, then pad to the max length."""
    y = [list(t) + [pad_id] for t in y]
    n = max(len(t) for t in y)
    y = [t + [pad_id] * (n - len(t)) for t in y]
    return torch.tensor(y, dtype=torch.int64, device=device)


def make_pad_mask(lengths: torch.Tensor, max_len: int = 0) -> torch.Tensor:
    """common.py:395-420 (True = padded position)."""
    assert lengths.ndim == 1, lengths.ndim
    max_len = max(int(max_len), int(lengths.max()))
    seq = torch.arange(0, max_len, device=lengths.device)
    return seq.unsqueeze(0).expand(lengths.size(0), max_len) >= lengths.unsqueeze(-1)


def speaker_turn_indices(tokens_padded: torch.Tensor, spk_a_id: int, spk_b_id: int,
                         pad_id: int) -> torch.Tensor:
    """ZipVoiceDialog.extract_spk_indices (zipvoice_dialog.py:118-125) as an int8
    map: 0 = speaker A, 1 = speaker B, -1 = padding."""
    turn = ((tokens_padded == spk_a_id) | (tokens_padded == spk_b_id)).long()
    spk = turn.cumsum(dim=1) % 2
    spk = torch.where(tokens_padded == pad_id, torch.full_like(spk, -1), spk)
    return spk.to(torch.int8)


def predict_features_lens(prompt_features_lens: torch.Tensor, prompt_tokens_lens: torch.Tensor,
                          tokens_lens: torch.Tensor, speed: float) -> torch.Tensor:
    """zipvoice.py:323-325: P + ceil(P / S_p * S_t / speed), in float32 as torch does
    for int64 / int64 true division."""
    r = prompt_features_lens.to(torch.float32) / prompt_tokens_lens.to(torch.float32)
    r = r * tokens_lens.to(torch.float32) / speed
    return prompt_features_lens + torch.ceil(r).to(torch.int64)

"""Sinusoidal positional embeddings — MI355X build of modules/position_embedding.py.

Same class, constructor and buffer (`_float_tensor`).  Positions are computed on the device
without the reference's host-side range buffer: position = t+1 where the token's feature 0 is
non-zero, 0 (padding) otherwise (make_positions, position_embedding.py:8-27, left_pad = 0).
"""
import math

import torch
import torch.nn as nn


def make_positions(tensor, padding_idx, left_pad):
    """(B, T) -> int64 positions; padding symbols (== padding_idx) keep padding_idx."""
    B, T = tensor.shape
    mask = tensor.ne(padding_idx)
    pos = torch.arange(padding_idx + 1, padding_idx + 1 + T, device=tensor.device).unsqueeze(0).expand(B, T)
    if left_pad:
        pos = pos - T + mask.long().sum(dim=1, keepdim=True)
    return torch.where(mask, pos, torch.full_like(pos, padding_idx))


class SinusoidalPositionalEmbedding(nn.Module):
    """Sinusoidal embeddings of any length (position_embedding.py:30-79)."""

    def __init__(self, embedding_dim, padding_idx=0, left_pad=0, init_size=128):
        super().__init__()
        self.embedding_dim = embedding_dim
        self.padding_idx = padding_idx
        self.left_pad = left_pad
        self.weights = dict()  # device -> table (not part of the state_dict, as in the reference)
        self.register_buffer('_float_tensor', torch.FloatTensor(1))

    @staticmethod
    def get_embedding(num_embeddings, embedding_dim, padding_idx=None):
        half = embedding_dim // 2
        freq = torch.exp(torch.arange(half, dtype=torch.float) * -(math.log(10000) / (half - 1)))
        ang = torch.arange(num_embeddings, dtype=torch.float).unsqueeze(1) * freq.unsqueeze(0)
        emb = torch.cat([torch.sin(ang), torch.cos(ang)], dim=1).view(num_embeddings, -1)
        if embedding_dim % 2 == 1:
            emb = torch.cat([emb, torch.zeros(num_embeddings, 1)], dim=1)
        if padding_idx is not None:
            emb[padding_idx, :] = 0
        return emb

    def forward(self, input):
        """input (B, T) -> (B, T, embedding_dim)."""
        bsz, seq_len = input.size()
        max_pos = self.padding_idx + 1 + seq_len
        key = input.device
        tab = self.weights.get(key)
        if tab is None or tab.size(0) < max_pos:
            tab = self.get_embedding(max_pos, self.embedding_dim, self.padding_idx).to(
                device=input.device, dtype=self._float_tensor.dtype)
            self.weights[key] = tab
        positions = make_positions(input, self.padding_idx, self.left_pad)
        return tab.index_select(0, positions.flatten()).view(bsz, seq_len, -1).detach()

    def max_positions(self):
        return int(1e5)

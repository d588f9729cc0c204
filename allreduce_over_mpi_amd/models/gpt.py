"""A small GPT-style decoder for data-parallel training over flexar.

Not a reference component (the reference ships no model code); it
is the workload that gradient allreduce serves: DDP buckets its gradients and the
flexar backend / comm hook reduces them over xGMI while backward continues.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class GPTConfig:
    vocab: int = 8192
    seq: int = 256
    d_model: int = 512
    n_layer: int = 6
    n_head: int = 8
    mlp_ratio: int = 4


PRESETS = {
    "gpt-tiny": GPTConfig(vocab=512, seq=64, d_model=128, n_layer=2, n_head=4),
    "gpt-small": GPTConfig(),
    "gpt-medium": GPTConfig(vocab=32000, seq=1024, d_model=1024, n_layer=24, n_head=16),
}


class Block(nn.Module):
    def __init__(self, c: GPTConfig):
        super().__init__()
        self.ln1 = nn.LayerNorm(c.d_model)
        self.qkv = nn.Linear(c.d_model, 3 * c.d_model)
        self.proj = nn.Linear(c.d_model, c.d_model)
        self.ln2 = nn.LayerNorm(c.d_model)
        self.fc1 = nn.Linear(c.d_model, c.mlp_ratio * c.d_model)
        self.fc2 = nn.Linear(c.mlp_ratio * c.d_model, c.d_model)
        self.n_head = c.n_head

    def forward(self, x):
        b, t, d = x.shape
        q, k, v = self.qkv(self.ln1(x)).split(d, dim=-1)
        h = self.n_head
        q, k, v = (z.view(b, t, h, d // h).transpose(1, 2) for z in (q, k, v))
        a = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        x = x + self.proj(a.transpose(1, 2).reshape(b, t, d))
        return x + self.fc2(F.gelu(self.fc1(self.ln2(x))))


class GPT(nn.Module):
    def __init__(self, c: GPTConfig):
        super().__init__()
        self.cfg = c
        self.tok = nn.Embedding(c.vocab, c.d_model)
        self.pos = nn.Embedding(c.seq, c.d_model)
        self.blocks = nn.ModuleList(Block(c) for _ in range(c.n_layer))
        self.ln = nn.LayerNorm(c.d_model)
        self.head = nn.Linear(c.d_model, c.vocab, bias=False)

    def forward(self, idx):
        t = idx.shape[1]
        x = self.tok(idx) + self.pos(torch.arange(t, device=idx.device))
        for blk in self.blocks:
            x = blk(x)
        return self.head(self.ln(x))

    def loss(self, idx, tgt):
        logits = self(idx)
        return F.cross_entropy(logits.reshape(-1, logits.shape[-1]).float(), tgt.reshape(-1))


def synthetic_batch(cfg: GPTConfig, batch: int, generator: torch.Generator, device):
    x = torch.randint(0, cfg.vocab, (batch, cfg.seq + 1), generator=generator).to(device)
    return x[:, :-1], x[:, 1:]

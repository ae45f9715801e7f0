"""Llama-3-8B architecture (hidden 4096, 32 layers, 32 heads / 8 KV heads, SwiGLU 14336, vocab
128256, RoPE theta 5e5, RMSNorm), local definition for QAT benchmarking. Every linear layer is a
`linear_cls(in, out)` module so a QAT linear (weight quantize-dequantize + matmul) can be plugged
in; random init N(0, 0.02) (seed)."""
import torch
from torch import nn


class RMSNorm(nn.Module):
    def __init__(self, dim, eps=1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        xf = x.float()
        return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)).to(x.dtype) * self.weight


def rope(x, cos, sin):
    x1, x2 = x[..., : x.shape[-1] // 2], x[..., x.shape[-1] // 2:]
    return x * cos + torch.cat([-x2, x1], dim=-1) * sin


class Attention(nn.Module):
    def __init__(self, linear_cls, dim=4096, heads=32, kv_heads=8):
        super().__init__()
        self.heads, self.kv_heads, self.hd = heads, kv_heads, dim // heads
        self.q_proj = linear_cls(dim, heads * self.hd)
        self.k_proj = linear_cls(dim, kv_heads * self.hd)
        self.v_proj = linear_cls(dim, kv_heads * self.hd)
        self.o_proj = linear_cls(heads * self.hd, dim)

    def forward(self, x, cos, sin):
        B, T, _ = x.shape
        q = self.q_proj(x).view(B, T, self.heads, self.hd).transpose(1, 2)
        k = self.k_proj(x).view(B, T, self.kv_heads, self.hd).transpose(1, 2)
        v = self.v_proj(x).view(B, T, self.kv_heads, self.hd).transpose(1, 2)
        q, k = rope(q, cos, sin), rope(k, cos, sin)
        rep = self.heads // self.kv_heads
        k, v = k.repeat_interleave(rep, dim=1), v.repeat_interleave(rep, dim=1)
        a = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True)
        return self.o_proj(a.transpose(1, 2).reshape(B, T, -1))


class MLP(nn.Module):
    def __init__(self, linear_cls, dim=4096, hidden=14336):
        super().__init__()
        self.gate_proj = linear_cls(dim, hidden)
        self.up_proj = linear_cls(dim, hidden)
        self.down_proj = linear_cls(hidden, dim)

    def forward(self, x):
        return self.down_proj(torch.nn.functional.silu(self.gate_proj(x)) * self.up_proj(x))


class Block(nn.Module):
    def __init__(self, linear_cls):
        super().__init__()
        self.input_layernorm = RMSNorm(4096)
        self.self_attn = Attention(linear_cls)
        self.post_attention_layernorm = RMSNorm(4096)
        self.mlp = MLP(linear_cls)

    def forward(self, x, cos, sin):
        x = x + self.self_attn(self.input_layernorm(x), cos, sin)
        return x + self.mlp(self.post_attention_layernorm(x))


class Llama(nn.Module):
    def __init__(self, linear_cls=nn.Linear, layers=32, vocab=128256):
        super().__init__()
        self.embed_tokens = nn.Embedding(vocab, 4096)
        self.layers = nn.ModuleList([Block(linear_cls) for _ in range(layers)])
        self.norm = RMSNorm(4096)
        self.lm_head = linear_cls(4096, vocab)

    def forward(self, ids):
        T = ids.shape[1]
        hd = 128
        inv = 1.0 / (500000.0 ** (torch.arange(0, hd, 2, device=ids.device).float() / hd))
        f = torch.outer(torch.arange(T, device=ids.device).float(), inv)
        emb = torch.cat([f, f], dim=-1)
        cos, sin = emb.cos()[None, None].to(torch.bfloat16), emb.sin()[None, None].to(torch.bfloat16)
        x = self.embed_tokens(ids)
        for blk in self.layers:
            x = blk(x, cos, sin)
        return self.lm_head(self.norm(x))

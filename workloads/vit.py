"""ViT-L/16 (224x224, 24 blocks, hidden 1024, MLP 4096, 16 heads), local definition with the
timm/torchvision layout: patch-embed conv, class token, learned position embedding, pre-LN
blocks (qkv / proj / fc1 / fc2 Linear layers, explicit scaled q @ k^T -> softmax -> @ v),
final LN, 1000-way head. Random init (seed). Every op QuantSim quantizes is a module
(activation_modules): per image 24 x (LN, qkv, q*scale, q@k^T, softmax, @v, proj, add, LN, fc1,
GELU, fc2, add) + patch conv, concat, pos add, LN, head -- about 122 M activation elements."""
import torch
from torch import nn


# Elementwise / matmul ops as modules (what aimet_torch's model preparer turns functional calls
# into, aimet_torch/elementwise_ops.py), so QuantizationSimModel places an output quantizer on each
class MatMul(nn.Module):
    def forward(self, a, b):
        return a @ b


class Mul(nn.Module):
    def forward(self, a, b):
        return a * b


class Add(nn.Module):
    def forward(self, a, b):
        return a + b


class Concat(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.dim = dim

    def forward(self, *xs):
        return torch.cat(xs, dim=self.dim)


class Block(nn.Module):
    """Pre-LN block with explicit attention (timm layout: q scaled before q @ k^T)."""

    def __init__(self, dim=1024, heads=16, mlp=4096):
        super().__init__()
        self.heads = heads
        self.scale = (dim // heads) ** -0.5
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.qkv = nn.Linear(dim, 3 * dim)
        self.q_scale = Mul()
        self.qk = MatMul()
        self.softmax = nn.Softmax(dim=-1)
        self.av = MatMul()
        self.proj = nn.Linear(dim, dim)
        self.add1 = Add()
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.fc1 = nn.Linear(dim, mlp)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(mlp, dim)
        self.add2 = Add()

    def forward(self, x):
        B, N, D = x.shape
        qkv = self.qkv(self.norm1(x)).view(B, N, 3, self.heads, D // self.heads).permute(2, 0, 3, 1, 4)
        q = self.q_scale(qkv[0], self.scale)
        attn = self.softmax(self.qk(q, qkv[1].transpose(-2, -1)))
        a = self.av(attn, qkv[2])
        x = self.add1(x, self.proj(a.transpose(1, 2).reshape(B, N, D)))
        return self.add2(x, self.fc2(self.act(self.fc1(self.norm2(x)))))


class ViT(nn.Module):
    def __init__(self, img=224, patch=16, dim=1024, depth=24, heads=16, mlp=4096, num_classes=1000):
        super().__init__()
        self.patch_embed = nn.Conv2d(3, dim, patch, stride=patch)
        n = (img // patch) ** 2
        self.cls_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos_embed = nn.Parameter(torch.randn(1, n + 1, dim) * 0.02)
        self.blocks = nn.ModuleList([Block(dim, heads, mlp) for _ in range(depth)])
        self.cat = Concat(1)
        self.pos_add = Add()
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        self.head = nn.Linear(dim, num_classes)

    def forward(self, x):
        x = self.patch_embed(x).flatten(2).transpose(1, 2)
        x = self.pos_add(self.cat(self.cls_token.expand(x.shape[0], -1, -1), x), self.pos_embed)
        for b in self.blocks:
            x = b(x)
        return self.head(self.norm(x)[:, 0])


# modules whose outputs carry an activation quantizer under QuantizationSimModel's default config
QUANTIZED_OUTPUT_TYPES = (nn.Conv2d, nn.Linear, nn.LayerNorm, nn.GELU, nn.Softmax, MatMul, Mul, Add, Concat)


def activation_modules(model):
    """Every module of `model` whose output QuantSim quantizes, in forward order."""
    return [m for m in model.modules() if isinstance(m, QUANTIZED_OUTPUT_TYPES)]


def vit_l16(seed=0, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    with torch.random.fork_rng(devices=[]):
        torch.manual_seed(seed)          # biases / LayerNorm: the default init, seeded too
        m = ViT()
    with torch.no_grad():
        for p in m.parameters():
            if p.dim() > 1:
                p.copy_(torch.randn(p.shape, generator=g) * (1.0 / p.shape[-1]) ** 0.5)
    return m.to(device).eval()

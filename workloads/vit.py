"""ViT-L/16 (224x224, 24 blocks, hidden 1024, MLP 4096, 16 heads), local definition with the
timm/torchvision layout: patch-embed conv, class token, learned position embedding, pre-LN
blocks (qkv / proj / fc1 / fc2 Linear layers), final LN, 1000-way head. Random init (seed)."""
import torch
from torch import nn


class Block(nn.Module):
    def __init__(self, dim=1024, heads=16, mlp=4096):
        super().__init__()
        self.heads = heads
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.qkv = nn.Linear(dim, 3 * dim)
        self.proj = nn.Linear(dim, dim)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.fc1 = nn.Linear(dim, mlp)
        self.act = nn.GELU()
        self.fc2 = nn.Linear(mlp, dim)

    def forward(self, x):
        B, N, D = x.shape
        qkv = self.qkv(self.norm1(x)).view(B, N, 3, self.heads, D // self.heads).permute(2, 0, 3, 1, 4)
        a = torch.nn.functional.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2])
        x = x + self.proj(a.transpose(1, 2).reshape(B, N, D))
        return x + self.fc2(self.act(self.fc1(self.norm2(x))))


class ViT(nn.Module):
    def __init__(self, img=224, patch=16, dim=1024, depth=24, heads=16, mlp=4096, num_classes=1000):
        super().__init__()
        self.patch_embed = nn.Conv2d(3, dim, patch, stride=patch)
        n = (img // patch) ** 2
        self.cls_token = nn.Parameter(torch.zeros(1, 1, dim))
        self.pos_embed = nn.Parameter(torch.randn(1, n + 1, dim) * 0.02)
        self.blocks = nn.ModuleList([Block(dim, heads, mlp) for _ in range(depth)])
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        self.head = nn.Linear(dim, num_classes)

    def forward(self, x):
        x = self.patch_embed(x).flatten(2).transpose(1, 2)
        x = torch.cat([self.cls_token.expand(x.shape[0], -1, -1), x], dim=1) + self.pos_embed
        for b in self.blocks:
            x = b(x)
        return self.head(self.norm(x)[:, 0])


def vit_l16(seed=0, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    m = ViT()
    with torch.no_grad():
        for p in m.parameters():
            if p.dim() > 1:
                p.copy_(torch.randn(p.shape, generator=g) * (1.0 / p.shape[-1]) ** 0.5)
    return m.to(device).eval()

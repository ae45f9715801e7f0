"""MobileNet-v2 (1.0, 224x224), local definition with batch norm already folded into the convs
(conv + bias, ReLU6), as AdaRound sees it after BN folding. Random init (seed)."""
import torch
from torch import nn


class InvertedResidual(nn.Module):
    def __init__(self, cin, cout, stride, expand):
        super().__init__()
        hidden = cin * expand
        self.use_res = stride == 1 and cin == cout
        layers = []
        if expand != 1:
            layers += [nn.Conv2d(cin, hidden, 1), nn.ReLU6()]
        layers += [nn.Conv2d(hidden, hidden, 3, stride, 1, groups=hidden), nn.ReLU6(),
                   nn.Conv2d(hidden, cout, 1)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.conv(x) if self.use_res else self.conv(x)


class MobileNetV2(nn.Module):
    CFG = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1)]

    def __init__(self, num_classes=1000):
        super().__init__()
        layers = [nn.Conv2d(3, 32, 3, 2, 1), nn.ReLU6()]
        cin = 32
        for t, c, n, s in self.CFG:
            for i in range(n):
                layers.append(InvertedResidual(cin, c, s if i == 0 else 1, t))
                cin = c
        layers += [nn.Conv2d(cin, 1280, 1), nn.ReLU6()]
        self.features = nn.Sequential(*layers)
        self.classifier = nn.Linear(1280, num_classes)

    def forward(self, x):
        x = self.features(x)
        return self.classifier(x.mean((2, 3)))


def mobilenet_v2(seed=0, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    m = MobileNetV2()
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, (nn.Conv2d, nn.Linear)):
                fan_in = mod.weight[0].numel()
                mod.weight.copy_(torch.randn(mod.weight.shape, generator=g) * (2.0 / fan_in) ** 0.5)
                mod.bias.copy_(torch.randn(mod.bias.shape, generator=g) * 0.01)
    return m.to(device).eval()

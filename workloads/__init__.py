"""Model graphs used as workloads by bench.py and the tests (written locally: no torchvision,
no pretrained weights; seeded random init)."""

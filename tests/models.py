"""Small training models for the optimizer goldens and the gloo tests (test code).

``TinyNet`` is the 2-layer MLP of the first optimizer golden. ``ResNet20`` is the
CIFAR ResNet-20 of BASELINE.json configs[0] (the reference builds it with
torchpack.mtpack.models.vision.resnet.resnet20, which is not installed here).
It is restated from the paper's description: 3 stages of 3 basic blocks at
16/32/64 channels, and parameter-free option-A shortcuts (stride-2 subsample,
then zero channel padding). Its parameter shapes equal
dgc.workloads.resnet20(): 269,722 parameters, 20 of them with dim > 1.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class TinyNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = nn.Linear(64, 128)
        self.fc2 = nn.Linear(128, 10)

    def forward(self, x):
        return self.fc2(torch.relu(self.fc1(x)))


class _Block(nn.Module):
    def __init__(self, cin, c, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, c, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(c)
        self.conv2 = nn.Conv2d(c, c, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(c)
        self.pad = c - cin
        self.stride = stride

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        sc = x
        if self.stride != 1 or self.pad:
            sc = x[:, :, ::self.stride, ::self.stride]
            sc = F.pad(sc, (0, 0, 0, 0, self.pad // 2, self.pad - self.pad // 2))
        return F.relu(out + sc)


class ResNet20(nn.Module):
    def __init__(self, num_classes=10):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 16, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(16)
        cin = 16
        for li, c in enumerate([16, 32, 64], start=1):
            blocks = []
            for b in range(3):
                blocks.append(_Block(cin, c, 2 if (b == 0 and li > 1) else 1))
                cin = c
            setattr(self, f"layer{li}", nn.Sequential(*blocks))
        self.fc = nn.Linear(64, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x):
        x = F.relu(self.bn1(self.conv1(x)))
        x = self.layer3(self.layer2(self.layer1(x)))
        x = F.adaptive_avg_pool2d(x, 1).flatten(1)
        return self.fc(x)

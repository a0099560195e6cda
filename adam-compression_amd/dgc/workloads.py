"""Gradient-shape sets of the BASELINE.json configurations.

The reference trains torchvision / torchpack models (configs/imagenet/*.py,
configs/cifar/*.py); the DGC path only ever sees their parameter SHAPES. The
reference applies compression to tensors with dim > 1 (train.py:137-140) and
sends the rest dense. The sets are generated here from the architectures'
definitions (torchvision is not installed), and checked against the published
totals:
  * ResNet-50: 25,557,032 parameters, 161 tensors, of them 54 compressed (25,502,912).
  * VGG-16-BN: 138,365,992 parameters, of them 16 compressed (138,344,128).
  * ResNet-20 (CIFAR, option-A shortcuts): 269,722 parameters, 20 compressed (268,336).
"""

__all__ = ["resnet50", "vgg16_bn", "resnet20", "flat", "split"]


def _bn(name, c):
    return [(f"{name}.weight", (c,)), (f"{name}.bias", (c,))]


def resnet50(num_classes=1000):
    shapes = [("conv1.weight", (64, 3, 7, 7))] + _bn("bn1", 64)
    inplanes = 64
    for li, (planes, blocks) in enumerate([(64, 3), (128, 4), (256, 6), (512, 3)], start=1):
        for b in range(blocks):
            p = f"layer{li}.{b}"
            shapes += [(f"{p}.conv1.weight", (planes, inplanes, 1, 1))] + _bn(f"{p}.bn1", planes)
            shapes += [(f"{p}.conv2.weight", (planes, planes, 3, 3))] + _bn(f"{p}.bn2", planes)
            shapes += [(f"{p}.conv3.weight", (planes * 4, planes, 1, 1))] + _bn(f"{p}.bn3", planes * 4)
            if b == 0:
                shapes += [(f"{p}.downsample.0.weight", (planes * 4, inplanes, 1, 1))]
                shapes += _bn(f"{p}.downsample.1", planes * 4)
            inplanes = planes * 4
    shapes += [("fc.weight", (num_classes, 2048)), ("fc.bias", (num_classes,))]
    return shapes


def vgg16_bn(num_classes=1000):
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
    shapes, cin, i = [], 3, 0
    for v in cfg:
        if v == "M":
            i += 1
            continue
        shapes += [(f"features.{i}.weight", (v, cin, 3, 3)), (f"features.{i}.bias", (v,))]
        shapes += _bn(f"features.{i + 1}", v)
        cin = v
        i += 3
    shapes += [("classifier.0.weight", (4096, 512 * 7 * 7)), ("classifier.0.bias", (4096,)),
               ("classifier.3.weight", (4096, 4096)), ("classifier.3.bias", (4096,)),
               ("classifier.6.weight", (num_classes, 4096)), ("classifier.6.bias", (num_classes,))]
    return shapes


def resnet20(num_classes=10):
    shapes = [("conv1.weight", (16, 3, 3, 3))] + _bn("bn1", 16)
    cin = 16
    for li, c in enumerate([16, 32, 64], start=1):
        for b in range(3):
            p = f"layer{li}.{b}"
            shapes += [(f"{p}.conv1.weight", (c, cin, 3, 3))] + _bn(f"{p}.bn1", c)
            shapes += [(f"{p}.conv2.weight", (c, c, 3, 3))] + _bn(f"{p}.bn2", c)
            cin = c
    shapes += [("fc.weight", (num_classes, 64)), ("fc.bias", (num_classes,))]
    return shapes


def numel(shape):
    n = 1
    for d in shape:
        n *= d
    return n


def split(shapes):
    """(compressed, dense) per the reference's dim > 1 rule (train.py:137-140)."""
    comp = [(n, s) for n, s in shapes if len(s) > 1]
    dense = [(n, s) for n, s in shapes if len(s) <= 1]
    return comp, dense


def flat(n):
    """A flat gradient bucket of n elements (BASELINE configs[3], configs[4])."""
    return [("bucket", (int(n),))]

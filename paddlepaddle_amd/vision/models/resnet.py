"""ResNet family. Reference: python/paddle/vision/models/resnet.py (same layer names so state dicts
line up: conv1/bn1/layer1..4/fc, BasicBlock/BottleneckBlock with downsample.0/.1).

MI355X: ``data_format="NHWC"`` keeps activations channels-last end-to-end (zero-copy views) so
MIOpen's NHWC convolution solvers run without relayout kernels between layers."""
from __future__ import annotations

from ... import nn


def _bn_act(bn, x, act="relu", residual=None, grad_sink=None):
    """bn(x) [+ residual] -> act as one fused pass (fused_bn_add_activation) when the norm layer
    supports it; any other norm layer composes the ops."""
    f = getattr(bn, "fused_forward", None)
    if f is not None:
        return f(x, act, residual, grad_sink) if grad_sink is not None else f(x, act, residual)
    y = bn(x)
    if residual is not None:
        y = y + residual
    return nn.functional.relu(y) if act == "relu" else y


class BasicBlock(nn.Layer):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None, data_format="NCHW"):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2D
        self.conv1 = nn.Conv2D(inplanes, planes, 3, padding=1, stride=stride, bias_attr=False,
                               data_format=data_format)
        self.bn1 = norm_layer(planes, data_format=data_format)
        self.relu = nn.ReLU()
        self.conv2 = nn.Conv2D(planes, planes, 3, padding=1, bias_attr=False, data_format=data_format)
        self.bn2 = norm_layer(planes, data_format=data_format)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        out = _bn_act(self.bn1, self.conv1(x))
        if self.downsample is not None:
            identity = self.downsample(x)
        return _bn_act(self.bn2, self.conv2(out), "relu", identity)


class BottleneckBlock(nn.Layer):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None, data_format="NCHW"):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2D
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = nn.Conv2D(inplanes, width, 1, bias_attr=False, data_format=data_format)
        self.bn1 = norm_layer(width, data_format=data_format)
        self.conv2 = nn.Conv2D(width, width, 3, padding=dilation, stride=stride, groups=groups, dilation=dilation,
                               bias_attr=False, data_format=data_format)
        self.bn2 = norm_layer(width, data_format=data_format)
        self.conv3 = nn.Conv2D(width, planes * self.expansion, 1, bias_attr=False, data_format=data_format)
        self.bn3 = norm_layer(planes * self.expansion, data_format=data_format)
        self.relu = nn.ReLU()
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x
        sink = None
        from ...ops.conv import residual_grad_producer, residual_grad_sink
        # x's two gradients are summed in conv1's GEMM epilogue: the other one comes from bn3 (identity shortcut)
        # or from the shortcut convolution (projection shortcut, residual_grad_producer)
        with residual_grad_sink() as sink:
            h = self.conv1(x)
        out = _bn_act(self.bn1, h)
        out = _bn_act(self.bn2, self.conv2(out))
        if self.downsample is not None:
            with residual_grad_producer(sink):
                identity = self.downsample(x)
            sink = None
        return _bn_act(self.bn3, self.conv3(out), "relu", identity, grad_sink=sink)


class ResNet(nn.Layer):
    def __init__(self, block, depth=50, width=64, num_classes=1000, with_pool=True, groups=1, data_format="NCHW"):
        super().__init__()
        layer_cfg = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3], 50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3]}
        layers = layer_cfg[depth]
        self.groups, self.base_width = groups, width
        self.num_classes, self.with_pool = num_classes, with_pool
        self.data_format = data_format
        self._norm_layer = nn.BatchNorm2D
        self.inplanes = 64
        self.dilation = 1
        self.conv1 = nn.Conv2D(3, self.inplanes, 7, stride=2, padding=3, bias_attr=False, data_format=data_format)
        self.bn1 = self._norm_layer(self.inplanes, data_format=data_format)
        self.relu = nn.ReLU()
        self.maxpool = nn.MaxPool2D(3, 2, 1, data_format=data_format)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D((1, 1), data_format=data_format)
        if num_classes > 0:
            self.fc = nn.Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, blocks, stride=1, dilate=False):
        norm_layer = self._norm_layer
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2D(self.inplanes, planes * block.expansion, 1, stride=stride, bias_attr=False,
                          data_format=self.data_format),
                norm_layer(planes * block.expansion, data_format=self.data_format))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width, 1, norm_layer,
                        self.data_format)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width,
                                norm_layer=norm_layer, data_format=self.data_format))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(_bn_act(self.bn1, self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            from ...tensor.manipulation import flatten
            x = flatten(x, 1)
            x = self.fc(x)
        return x


def _resnet(block, depth, pretrained=False, **kwargs):
    if pretrained:
        raise ValueError("pretrained weights are not available offline")
    return ResNet(block, depth, **kwargs)


def resnet18(pretrained=False, **kwargs):
    return _resnet(BasicBlock, 18, pretrained, **kwargs)


def resnet34(pretrained=False, **kwargs):
    return _resnet(BasicBlock, 34, pretrained, **kwargs)


def resnet50(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 50, pretrained, **kwargs)


def resnet101(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 101, pretrained, **kwargs)


def resnet152(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 152, pretrained, **kwargs)


def resnext50_32x4d(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 50, pretrained, width=4, groups=32, **kwargs)


def resnext50_64x4d(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 50, pretrained, width=4, groups=64, **kwargs)


def resnext101_32x4d(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 101, pretrained, width=4, groups=32, **kwargs)


def resnext101_64x4d(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 101, pretrained, width=4, groups=64, **kwargs)


def resnext152_32x4d(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 152, pretrained, width=4, groups=32, **kwargs)


def resnext152_64x4d(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 152, pretrained, width=4, groups=64, **kwargs)


def wide_resnet50_2(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 50, pretrained, width=128, **kwargs)


def wide_resnet101_2(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 101, pretrained, width=128, **kwargs)

"""MobileNet V1 / V2 / V3 and ShuffleNetV2. Reference: python/paddle/vision/models/{mobilenetv1,
mobilenetv2,mobilenetv3,shufflenetv2}.py. Depthwise convolutions go to MIOpen's grouped conv."""
from __future__ import annotations

from ... import nn
from ...tensor.manipulation import flatten, concat, reshape, transpose, split
from .vgg import _no_pretrained


def _make_divisible(v, divisor=8, min_value=None):
    min_value = min_value or divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


class ConvBNLayer(nn.Layer):
    def __init__(self, cin, cout, k, stride=1, padding=None, groups=1, act=nn.ReLU):
        super().__init__()
        self.conv = nn.Conv2D(cin, cout, k, stride=stride, padding=(k - 1) // 2 if padding is None else padding,
                              groups=groups, bias_attr=False)
        self.bn = nn.BatchNorm2D(cout)
        self.act = act() if act is not None else None

    def forward(self, x):
        x = self.bn(self.conv(x))
        return self.act(x) if self.act is not None else x


# ---------------------------------------------------------------------------- V1
class _DepthwiseSeparable(nn.Layer):
    def __init__(self, cin, c1, c2, groups, stride, scale):
        super().__init__()
        self.dw = ConvBNLayer(cin, int(c1 * scale), 3, stride, groups=int(groups * scale))
        self.pw = ConvBNLayer(int(c1 * scale), int(c2 * scale), 1)

    def forward(self, x):
        return self.pw(self.dw(x))


class MobileNetV1(nn.Layer):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        self.conv1 = ConvBNLayer(3, int(32 * scale), 3, 2)
        cfg = [(32, 32, 64, 32, 1), (64, 64, 128, 64, 2), (128, 128, 128, 128, 1), (128, 128, 256, 128, 2),
               (256, 256, 256, 256, 1), (256, 256, 512, 256, 2)] + [(512, 512, 512, 512, 1)] * 5 + \
              [(512, 512, 1024, 512, 2), (1024, 1024, 1024, 1024, 1)]
        self.dwsl = nn.Sequential(*[_DepthwiseSeparable(int(a * scale), b, c, g, s, scale) for a, b, c, g, s in cfg])
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.fc = nn.Linear(int(1024 * scale), num_classes)

    def forward(self, x):
        x = self.dwsl(self.conv1(x))
        if self.with_pool:
            x = self.pool2d_avg(x)
        if self.num_classes > 0:
            x = self.fc(flatten(x, 1))
        return x


def mobilenet_v1(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV1(scale=scale, **kw)


# ---------------------------------------------------------------------------- V2
class InvertedResidual(nn.Layer):
    def __init__(self, cin, cout, stride, expand_ratio):
        super().__init__()
        hidden = int(round(cin * expand_ratio))
        self.use_res = stride == 1 and cin == cout
        layers = []
        if expand_ratio != 1:
            layers.append(ConvBNLayer(cin, hidden, 1, act=nn.ReLU6))
        layers += [ConvBNLayer(hidden, hidden, 3, stride, groups=hidden, act=nn.ReLU6),
                   ConvBNLayer(hidden, cout, 1, act=None)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.conv(x) if self.use_res else self.conv(x)


class MobileNetV2(nn.Layer):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        cin = _make_divisible(32 * scale)
        self.last_channel = _make_divisible(1280 * max(1.0, scale))
        cfg = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2),
               (6, 320, 1, 1)]
        feats = [ConvBNLayer(3, cin, 3, 2, act=nn.ReLU6)]
        for t, c, n, s in cfg:
            cout = _make_divisible(c * scale)
            for i in range(n):
                feats.append(InvertedResidual(cin, cout, s if i == 0 else 1, t))
                cin = cout
        feats.append(ConvBNLayer(cin, self.last_channel, 1, act=nn.ReLU6))
        self.features = nn.Sequential(*feats)
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Dropout(0.2), nn.Linear(self.last_channel, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool2d_avg(x)
        if self.num_classes > 0:
            x = self.classifier(flatten(x, 1))
        return x


def mobilenet_v2(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV2(scale=scale, **kw)


# ---------------------------------------------------------------------------- V3
class _SE(nn.Layer):
    def __init__(self, c, r=4):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2D(1)
        mid = _make_divisible(c // r)
        self.conv1 = nn.Conv2D(c, mid, 1)
        self.relu = nn.ReLU()
        self.conv2 = nn.Conv2D(mid, c, 1)
        self.hardsigmoid = nn.Hardsigmoid()

    def forward(self, x):
        s = self.hardsigmoid(self.conv2(self.relu(self.conv1(self.avg_pool(x)))))
        return x * s


class _V3Block(nn.Layer):
    def __init__(self, cin, k, exp, cout, use_se, act, stride):
        super().__init__()
        A = nn.Hardswish if act == "hardswish" else nn.ReLU
        self.use_res = stride == 1 and cin == cout
        layers = []
        if exp != cin:
            layers.append(ConvBNLayer(cin, exp, 1, act=A))
        layers.append(ConvBNLayer(exp, exp, k, stride, groups=exp, act=A))
        if use_se:
            layers.append(_SE(exp))
        layers.append(ConvBNLayer(exp, cout, 1, act=None))
        self.block = nn.Sequential(*layers)

    def forward(self, x):
        y = self.block(x)
        return x + y if self.use_res else y


class MobileNetV3(nn.Layer):
    def __init__(self, config, last_channel, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        cin = _make_divisible(16 * scale)
        self.conv = ConvBNLayer(3, cin, 3, 2, act=nn.Hardswish)
        blocks = []
        for k, exp, c, se, act, s in config:
            cout = _make_divisible(c * scale)
            blocks.append(_V3Block(cin, k, _make_divisible(exp * scale), cout, se, act, s))
            cin = cout
        self.blocks = nn.Sequential(*blocks)
        lc = _make_divisible(config[-1][1] * scale)
        self.lastconv = ConvBNLayer(cin, lc, 1, act=nn.Hardswish)
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Linear(lc, last_channel), nn.Hardswish(), nn.Dropout(0.2),
                                            nn.Linear(last_channel, num_classes))

    def forward(self, x):
        x = self.lastconv(self.blocks(self.conv(x)))
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            x = self.classifier(flatten(x, 1))
        return x


_V3_SMALL = [(3, 16, 16, True, "relu", 2), (3, 72, 24, False, "relu", 2), (3, 88, 24, False, "relu", 1),
             (5, 96, 40, True, "hardswish", 2), (5, 240, 40, True, "hardswish", 1),
             (5, 240, 40, True, "hardswish", 1), (5, 120, 48, True, "hardswish", 1),
             (5, 144, 48, True, "hardswish", 1), (5, 288, 96, True, "hardswish", 2),
             (5, 576, 96, True, "hardswish", 1), (5, 576, 96, True, "hardswish", 1)]
_V3_LARGE = [(3, 16, 16, False, "relu", 1), (3, 64, 24, False, "relu", 2), (3, 72, 24, False, "relu", 1),
             (5, 72, 40, True, "relu", 2), (5, 120, 40, True, "relu", 1), (5, 120, 40, True, "relu", 1),
             (3, 240, 80, False, "hardswish", 2), (3, 200, 80, False, "hardswish", 1),
             (3, 184, 80, False, "hardswish", 1), (3, 184, 80, False, "hardswish", 1),
             (3, 480, 112, True, "hardswish", 1), (3, 672, 112, True, "hardswish", 1),
             (5, 672, 160, True, "hardswish", 2), (5, 960, 160, True, "hardswish", 1),
             (5, 960, 160, True, "hardswish", 1)]


class MobileNetV3Small(MobileNetV3):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__(_V3_SMALL, 1024, scale, num_classes, with_pool)


class MobileNetV3Large(MobileNetV3):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__(_V3_LARGE, 1280, scale, num_classes, with_pool)


def mobilenet_v3_small(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV3Small(scale=scale, **kw)


def mobilenet_v3_large(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV3Large(scale=scale, **kw)


# ---------------------------------------------------------------------------- ShuffleNetV2
def channel_shuffle(x, groups):
    b, c, h, w = x.shape
    x = reshape(x, [b, groups, c // groups, h, w])
    x = transpose(x, [0, 2, 1, 3, 4])
    return reshape(x, [b, c, h, w])


class _ShuffleUnit(nn.Layer):
    def __init__(self, cin, cout, stride, act):
        super().__init__()
        self.stride = stride
        branch = cout // 2
        if stride == 1:
            self.branch2 = nn.Sequential(ConvBNLayer(branch, branch, 1, act=act),
                                         ConvBNLayer(branch, branch, 3, 1, groups=branch, act=None),
                                         ConvBNLayer(branch, branch, 1, act=act))
        else:
            self.branch1 = nn.Sequential(ConvBNLayer(cin, cin, 3, stride, groups=cin, act=None),
                                         ConvBNLayer(cin, branch, 1, act=act))
            self.branch2 = nn.Sequential(ConvBNLayer(cin, branch, 1, act=act),
                                         ConvBNLayer(branch, branch, 3, stride, groups=branch, act=None),
                                         ConvBNLayer(branch, branch, 1, act=act))

    def forward(self, x):
        if self.stride == 1:
            x1, x2 = split(x, 2, axis=1)
            out = concat([x1, self.branch2(x2)], axis=1)
        else:
            out = concat([self.branch1(x), self.branch2(x)], axis=1)
        return channel_shuffle(out, 2)


class ShuffleNetV2(nn.Layer):
    _CH = {0.25: [24, 24, 48, 96, 512], 0.33: [24, 32, 64, 128, 512], 0.5: [24, 48, 96, 192, 1024],
           1.0: [24, 116, 232, 464, 1024], 1.5: [24, 176, 352, 704, 1024], 2.0: [24, 244, 488, 976, 2048]}

    def __init__(self, scale=1.0, act="relu", num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        A = {"relu": nn.ReLU, "swish": nn.Swish}[act]
        ch = self._CH[scale]
        self.conv1 = ConvBNLayer(3, ch[0], 3, 2, act=A)
        self.max_pool = nn.MaxPool2D(3, 2, padding=1)
        units, cin = [], ch[0]
        for stage, reps in enumerate([4, 8, 4]):
            cout = ch[stage + 1]
            for i in range(reps):
                units.append(_ShuffleUnit(cin, cout, 2 if i == 0 else 1, A))
                cin = cout
        self.blocks = nn.Sequential(*units)
        self.last_conv = ConvBNLayer(cin, ch[-1], 1, act=A)
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.fc = nn.Linear(ch[-1], num_classes)

    def forward(self, x):
        x = self.last_conv(self.blocks(self.max_pool(self.conv1(x))))
        if self.with_pool:
            x = self.pool2d_avg(x)
        if self.num_classes > 0:
            x = self.fc(flatten(x, 1))
        return x


def _shufflenet(scale, act="relu", pretrained=False, **kw):
    _no_pretrained(pretrained)
    return ShuffleNetV2(scale, act, **kw)


def shufflenet_v2_x0_25(pretrained=False, **kw):
    return _shufflenet(0.25, pretrained=pretrained, **kw)


def shufflenet_v2_x0_33(pretrained=False, **kw):
    return _shufflenet(0.33, pretrained=pretrained, **kw)


def shufflenet_v2_x0_5(pretrained=False, **kw):
    return _shufflenet(0.5, pretrained=pretrained, **kw)


def shufflenet_v2_x1_0(pretrained=False, **kw):
    return _shufflenet(1.0, pretrained=pretrained, **kw)


def shufflenet_v2_x1_5(pretrained=False, **kw):
    return _shufflenet(1.5, pretrained=pretrained, **kw)


def shufflenet_v2_x2_0(pretrained=False, **kw):
    return _shufflenet(2.0, pretrained=pretrained, **kw)


def shufflenet_v2_swish(pretrained=False, **kw):
    return _shufflenet(1.0, "swish", pretrained=pretrained, **kw)

"""DenseNet, GoogLeNet, InceptionV3. Reference: python/paddle/vision/models/{densenet,googlenet,
inceptionv3}.py."""
from __future__ import annotations

from ... import nn
from ...tensor.manipulation import flatten, concat
from .mobilenet import ConvBNLayer
from .vgg import _no_pretrained


# ---------------------------------------------------------------------------- DenseNet
class _DenseLayer(nn.Layer):
    def __init__(self, cin, growth, bn_size, dropout):
        super().__init__()
        self.bn1 = nn.BatchNorm2D(cin)
        self.conv1 = nn.Conv2D(cin, bn_size * growth, 1, bias_attr=False)
        self.bn2 = nn.BatchNorm2D(bn_size * growth)
        self.conv2 = nn.Conv2D(bn_size * growth, growth, 3, padding=1, bias_attr=False)
        self.relu = nn.ReLU()
        self.dropout = nn.Dropout(dropout) if dropout else None

    def forward(self, x):
        y = self.conv1(self.relu(self.bn1(x)))
        y = self.conv2(self.relu(self.bn2(y)))
        if self.dropout is not None:
            y = self.dropout(y)
        return concat([x, y], axis=1)


class _Transition(nn.Layer):
    def __init__(self, cin, cout):
        super().__init__()
        self.bn = nn.BatchNorm2D(cin)
        self.relu = nn.ReLU()
        self.conv = nn.Conv2D(cin, cout, 1, bias_attr=False)
        self.pool = nn.AvgPool2D(2, 2)

    def forward(self, x):
        return self.pool(self.conv(self.relu(self.bn(x))))


class DenseNet(nn.Layer):
    _CFG = {121: (64, 32, [6, 12, 24, 16]), 161: (96, 48, [6, 12, 36, 24]), 169: (64, 32, [6, 12, 32, 32]),
            201: (64, 32, [6, 12, 48, 32]), 264: (64, 32, [6, 12, 64, 48])}

    def __init__(self, layers=121, bn_size=4, dropout=0.0, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        init_c, growth, blocks = self._CFG[layers]
        feats = [nn.Conv2D(3, init_c, 7, stride=2, padding=3, bias_attr=False), nn.BatchNorm2D(init_c), nn.ReLU(),
                 nn.MaxPool2D(3, 2, padding=1)]
        c = init_c
        for i, n in enumerate(blocks):
            for _ in range(n):
                feats.append(_DenseLayer(c, growth, bn_size, dropout))
                c += growth
            if i != len(blocks) - 1:
                feats.append(_Transition(c, c // 2))
                c //= 2
        feats += [nn.BatchNorm2D(c), nn.ReLU()]
        self.features = nn.Sequential(*feats)
        if with_pool:
            self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.out = nn.Linear(c, num_classes)

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool2d_avg(x)
        if self.num_classes > 0:
            x = self.out(flatten(x, 1))
        return x


def _densenet(n, pretrained, **kw):
    _no_pretrained(pretrained)
    return DenseNet(n, **kw)


def densenet121(pretrained=False, **kw):
    return _densenet(121, pretrained, **kw)


def densenet161(pretrained=False, **kw):
    return _densenet(161, pretrained, **kw)


def densenet169(pretrained=False, **kw):
    return _densenet(169, pretrained, **kw)


def densenet201(pretrained=False, **kw):
    return _densenet(201, pretrained, **kw)


def densenet264(pretrained=False, **kw):
    return _densenet(264, pretrained, **kw)


# ---------------------------------------------------------------------------- GoogLeNet
class _Inception(nn.Layer):
    def __init__(self, cin, c1, c3r, c3, c5r, c5, proj):
        super().__init__()
        self.b1 = ConvBNLayer(cin, c1, 1)
        self.b2 = nn.Sequential(ConvBNLayer(cin, c3r, 1), ConvBNLayer(c3r, c3, 3))
        self.b3 = nn.Sequential(ConvBNLayer(cin, c5r, 1), ConvBNLayer(c5r, c5, 5))
        self.b4 = nn.Sequential(nn.MaxPool2D(3, 1, padding=1), ConvBNLayer(cin, proj, 1))

    def forward(self, x):
        return concat([self.b1(x), self.b2(x), self.b3(x), self.b4(x)], axis=1)


class GoogLeNet(nn.Layer):
    """Returns (out, aux1, aux2) like the reference."""

    def __init__(self, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        self.stem = nn.Sequential(ConvBNLayer(3, 64, 7, 2), nn.MaxPool2D(3, 2, padding=1), ConvBNLayer(64, 64, 1),
                                  ConvBNLayer(64, 192, 3), nn.MaxPool2D(3, 2, padding=1))
        self.i3a = _Inception(192, 64, 96, 128, 16, 32, 32)
        self.i3b = _Inception(256, 128, 128, 192, 32, 96, 64)
        self.pool3 = nn.MaxPool2D(3, 2, padding=1)
        self.i4a = _Inception(480, 192, 96, 208, 16, 48, 64)
        self.i4b = _Inception(512, 160, 112, 224, 24, 64, 64)
        self.i4c = _Inception(512, 128, 128, 256, 24, 64, 64)
        self.i4d = _Inception(512, 112, 144, 288, 32, 64, 64)
        self.i4e = _Inception(528, 256, 160, 320, 32, 128, 128)
        self.pool4 = nn.MaxPool2D(3, 2, padding=1)
        self.i5a = _Inception(832, 256, 160, 320, 32, 128, 128)
        self.i5b = _Inception(832, 384, 192, 384, 48, 128, 128)
        if with_pool:
            self.pool5 = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.dropout = nn.Dropout(0.4)
            self.fc = nn.Linear(1024, num_classes)
            self.aux1 = self._aux(512, num_classes)
            self.aux2 = self._aux(528, num_classes)

    @staticmethod
    def _aux(cin, n):
        return nn.Sequential(nn.AdaptiveAvgPool2D(4), ConvBNLayer(cin, 128, 1), nn.Flatten(),
                             nn.Linear(2048, 1024), nn.ReLU(), nn.Dropout(0.7), nn.Linear(1024, n))

    def forward(self, x):
        x = self.pool3(self.i3b(self.i3a(self.stem(x))))
        a = self.i4a(x)
        x = self.i4c(self.i4b(a))
        b = self.i4d(x)
        x = self.pool4(self.i4e(b))
        x = self.i5b(self.i5a(x))
        if self.with_pool:
            x = self.pool5(x)
        if self.num_classes > 0:
            out = self.fc(self.dropout(flatten(x, 1)))
            return out, self.aux1(a), self.aux2(b)
        return x


def googlenet(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return GoogLeNet(**kw)


# ---------------------------------------------------------------------------- InceptionV3
class _IncA(nn.Layer):
    def __init__(self, cin, pool_c):
        super().__init__()
        self.b1 = ConvBNLayer(cin, 64, 1)
        self.b5 = nn.Sequential(ConvBNLayer(cin, 48, 1), ConvBNLayer(48, 64, 5))
        self.b3 = nn.Sequential(ConvBNLayer(cin, 64, 1), ConvBNLayer(64, 96, 3), ConvBNLayer(96, 96, 3))
        self.bp = nn.Sequential(nn.AvgPool2D(3, 1, padding=1, exclusive=False), ConvBNLayer(cin, pool_c, 1))

    def forward(self, x):
        return concat([self.b1(x), self.b5(x), self.b3(x), self.bp(x)], axis=1)


class _IncB(nn.Layer):
    def __init__(self, cin):
        super().__init__()
        self.b3 = ConvBNLayer(cin, 384, 3, 2, padding=0)
        self.b33 = nn.Sequential(ConvBNLayer(cin, 64, 1), ConvBNLayer(64, 96, 3),
                                 ConvBNLayer(96, 96, 3, 2, padding=0))
        self.bp = nn.MaxPool2D(3, 2)

    def forward(self, x):
        return concat([self.b3(x), self.b33(x), self.bp(x)], axis=1)


class _IncC(nn.Layer):
    def __init__(self, cin, c7):
        super().__init__()

        def c17(a, b):
            return ConvBNLayer(a, b, (1, 7), padding=(0, 3))

        def c71(a, b):
            return ConvBNLayer(a, b, (7, 1), padding=(3, 0))
        self.b1 = ConvBNLayer(cin, 192, 1)
        self.b7 = nn.Sequential(ConvBNLayer(cin, c7, 1), c17(c7, c7), c71(c7, 192))
        self.b77 = nn.Sequential(ConvBNLayer(cin, c7, 1), c71(c7, c7), c17(c7, c7), c71(c7, c7), c17(c7, 192))
        self.bp = nn.Sequential(nn.AvgPool2D(3, 1, padding=1, exclusive=False), ConvBNLayer(cin, 192, 1))

    def forward(self, x):
        return concat([self.b1(x), self.b7(x), self.b77(x), self.bp(x)], axis=1)


class _IncD(nn.Layer):
    def __init__(self, cin):
        super().__init__()
        self.b3 = nn.Sequential(ConvBNLayer(cin, 192, 1), ConvBNLayer(192, 320, 3, 2, padding=0))
        self.b7 = nn.Sequential(ConvBNLayer(cin, 192, 1), ConvBNLayer(192, 192, (1, 7), padding=(0, 3)),
                                ConvBNLayer(192, 192, (7, 1), padding=(3, 0)), ConvBNLayer(192, 192, 3, 2, padding=0))
        self.bp = nn.MaxPool2D(3, 2)

    def forward(self, x):
        return concat([self.b3(x), self.b7(x), self.bp(x)], axis=1)


class _IncE(nn.Layer):
    def __init__(self, cin):
        super().__init__()
        self.b1 = ConvBNLayer(cin, 320, 1)
        self.b3 = ConvBNLayer(cin, 384, 1)
        self.b3a = ConvBNLayer(384, 384, (1, 3), padding=(0, 1))
        self.b3b = ConvBNLayer(384, 384, (3, 1), padding=(1, 0))
        self.b33 = nn.Sequential(ConvBNLayer(cin, 448, 1), ConvBNLayer(448, 384, 3))
        self.b33a = ConvBNLayer(384, 384, (1, 3), padding=(0, 1))
        self.b33b = ConvBNLayer(384, 384, (3, 1), padding=(1, 0))
        self.bp = nn.Sequential(nn.AvgPool2D(3, 1, padding=1, exclusive=False), ConvBNLayer(cin, 192, 1))

    def forward(self, x):
        a = self.b3(x)
        b = self.b33(x)
        return concat([self.b1(x), self.b3a(a), self.b3b(a), self.b33a(b), self.b33b(b), self.bp(x)], axis=1)


class InceptionV3(nn.Layer):
    def __init__(self, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        self.stem = nn.Sequential(ConvBNLayer(3, 32, 3, 2, padding=0), ConvBNLayer(32, 32, 3, padding=0),
                                  ConvBNLayer(32, 64, 3), nn.MaxPool2D(3, 2), ConvBNLayer(64, 80, 1),
                                  ConvBNLayer(80, 192, 3, padding=0), nn.MaxPool2D(3, 2))
        self.blocks = nn.Sequential(_IncA(192, 32), _IncA(256, 64), _IncA(288, 64), _IncB(288),
                                    _IncC(768, 128), _IncC(768, 160), _IncC(768, 160), _IncC(768, 192),
                                    _IncD(768), _IncE(1280), _IncE(2048))
        if with_pool:
            self.avg_pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.dropout = nn.Dropout(0.2)
            self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        x = self.blocks(self.stem(x))
        if self.with_pool:
            x = self.avg_pool(x)
        if self.num_classes > 0:
            x = self.fc(self.dropout(flatten(x, 1)))
        return x


def inception_v3(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return InceptionV3(**kw)

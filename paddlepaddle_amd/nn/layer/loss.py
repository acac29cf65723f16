"""Loss layers. Reference: python/paddle/nn/layer/loss.py."""
from __future__ import annotations

from .. import functional as F
from .layers import Layer


class CrossEntropyLoss(Layer):
    def __init__(self, weight=None, ignore_index=-100, reduction="mean", soft_label=False, axis=-1,
                 use_softmax=True, label_smoothing=0.0, name=None):
        super().__init__()
        self.weight, self.ignore_index, self.reduction = weight, ignore_index, reduction
        self.soft_label, self.axis, self.use_softmax = soft_label, axis, use_softmax
        self.label_smoothing = label_smoothing

    def forward(self, input, label):
        return F.cross_entropy(input, label, self.weight, self.ignore_index, self.reduction, self.soft_label,
                               self.axis, self.use_softmax, self.label_smoothing)


def _loss_layer(name, fn, params):
    names = [p for p, _ in params]
    defaults = dict(params)

    def __init__(self, *args, name=None, **kwargs):
        Layer.__init__(self)
        vals = dict(zip(names, args))
        for k in names:
            setattr(self, "_" + k, kwargs.get(k, vals.get(k, defaults[k])))

    def forward(self, *inputs):
        return fn(*inputs, **{k: getattr(self, "_" + k) for k in names})

    return type(name, (Layer,), {"__init__": __init__, "forward": forward})


MSELoss = _loss_layer("MSELoss", F.mse_loss, (("reduction", "mean"),))
L1Loss = _loss_layer("L1Loss", F.l1_loss, (("reduction", "mean"),))
NLLLoss = _loss_layer("NLLLoss", F.nll_loss, (("weight", None), ("ignore_index", -100), ("reduction", "mean")))
BCELoss = _loss_layer("BCELoss", F.binary_cross_entropy, (("weight", None), ("reduction", "mean")))
BCEWithLogitsLoss = _loss_layer("BCEWithLogitsLoss", F.binary_cross_entropy_with_logits,
                                (("weight", None), ("reduction", "mean"), ("pos_weight", None)))
KLDivLoss = _loss_layer("KLDivLoss", F.kl_div, (("reduction", "mean"), ("log_target", False)))
SmoothL1Loss = _loss_layer("SmoothL1Loss", F.smooth_l1_loss, (("reduction", "mean"), ("delta", 1.0)))
HuberLoss = _loss_layer("HuberLoss", F.huber_loss, (("reduction", "mean"), ("delta", 1.0)))
MarginRankingLoss = _loss_layer("MarginRankingLoss", F.margin_ranking_loss, (("margin", 0.0), ("reduction", "mean")))
HingeEmbeddingLoss = _loss_layer("HingeEmbeddingLoss", F.hinge_embedding_loss,
                                 (("margin", 1.0), ("reduction", "mean")))
CosineEmbeddingLoss = _loss_layer("CosineEmbeddingLoss", F.cosine_embedding_loss,
                                  (("margin", 0), ("reduction", "mean")))
TripletMarginLoss = _loss_layer("TripletMarginLoss", F.triplet_margin_loss,
                                (("margin", 1.0), ("p", 2.0), ("epsilon", 1e-6), ("swap", False),
                                 ("reduction", "mean")))
TripletMarginWithDistanceLoss = _loss_layer("TripletMarginWithDistanceLoss", F.triplet_margin_with_distance_loss,
                                            (("distance_function", None), ("margin", 1.0), ("swap", False),
                                             ("reduction", "mean")))
MultiLabelSoftMarginLoss = _loss_layer("MultiLabelSoftMarginLoss", F.multi_label_soft_margin_loss,
                                       (("weight", None), ("reduction", "mean")))
MultiMarginLoss = _loss_layer("MultiMarginLoss", F.multi_margin_loss,
                              (("p", 1), ("margin", 1.0), ("weight", None), ("reduction", "mean")))
SoftMarginLoss = _loss_layer("SoftMarginLoss", F.soft_margin_loss, (("reduction", "mean"),))
PoissonNLLLoss = _loss_layer("PoissonNLLLoss", F.poisson_nll_loss,
                             (("log_input", True), ("full", False), ("epsilon", 1e-8), ("reduction", "mean")))
GaussianNLLLoss = _loss_layer("GaussianNLLLoss", F.gaussian_nll_loss,
                              (("full", False), ("epsilon", 1e-6), ("reduction", "mean")))
CTCLoss = _loss_layer("CTCLoss", F.ctc_loss, (("blank", 0), ("reduction", "mean")))

"""paddle.distribution. Reference: python/paddle/distribution/__init__.py.

Densities, moments, entropies, CDFs and KL divergences are this package's own formulas on device tensors
(one module per distribution, like the reference); sampling uses the device RNG (paddle.seed) with
reparameterised samplers where the distribution has one."""
from . import transform  # noqa: F401
from .bernoulli import Bernoulli
from .beta import Beta
from .binomial import Binomial
from .categorical import Categorical
from .cauchy import Cauchy
from .chi2 import Chi2
from .continuous_bernoulli import ContinuousBernoulli
from .dirichlet import Dirichlet
from .distribution import Distribution
from .exponential import Exponential
from .exponential_family import ExponentialFamily
from .gamma import Gamma
from .geometric import Geometric
from .gumbel import Gumbel
from .independent import Independent
from .kl import kl_divergence, register_kl
from .laplace import Laplace
from .lkj_cholesky import LKJCholesky
from .lognormal import LogNormal
from .multinomial import Multinomial
from .multivariate_normal import MultivariateNormal
from .normal import Normal
from .poisson import Poisson
from .student_t import StudentT
from .transform import (AbsTransform, AffineTransform, ChainTransform, ExpTransform,  # noqa: F401
                        IndependentTransform, PowerTransform, ReshapeTransform, SigmoidTransform, SoftmaxTransform,
                        StackTransform, StickBreakingTransform, TanhTransform, Transform)
from .transformed_distribution import TransformedDistribution
from .uniform import Uniform

__all__ = ["Bernoulli", "Beta", "Categorical", "Cauchy", "Chi2", "ContinuousBernoulli", "Dirichlet", "Distribution",
           "Exponential", "ExponentialFamily", "Multinomial", "MultivariateNormal", "Normal", "Uniform",
           "kl_divergence", "register_kl", "Independent", "TransformedDistribution", "Laplace", "LogNormal",
           "LKJCholesky", "Gamma", "Gumbel", "Geometric", "Binomial", "Poisson", "StudentT"]
__all__ += transform.__all__

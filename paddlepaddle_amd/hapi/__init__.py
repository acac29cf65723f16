"""paddle.hapi (in progress)."""


class Model:
    pass


def summary(*a, **k):
    raise NotImplementedError


def flops(*a, **k):
    raise NotImplementedError

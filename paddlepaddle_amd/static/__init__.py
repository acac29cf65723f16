"""paddle.static (filled in by static/program.py)."""


class _StaticMode:
    enabled = False


_static_mode = _StaticMode()


def enable_static():
    _static_mode.enabled = True


def disable_static(place=None):
    _static_mode.enabled = False

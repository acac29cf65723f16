"""paddle.static.amp (reference python/paddle/static/amp/): mixed precision for static programs. Our
static programs are recorded from the same ops as dygraph, so the dygraph AMP machinery (auto_cast lists,
decorate with master weights, dynamic loss scaling) applies unchanged."""
import contextlib

from ..amp import auto_cast, decorate as _decorate, GradScaler, is_float16_supported, is_bfloat16_supported  # noqa


class AutoMixedPrecisionLists:
    """White / black op lists for static AMP (names of ops forced to low / full precision)."""

    def __init__(self, custom_white_list=None, custom_black_list=None, custom_black_varnames=None, dtype="float16"):
        from ..amp.state import WHITE_LIST, BLACK_LIST
        self.white_list = set(WHITE_LIST) | set(custom_white_list or ())
        self.black_list = (set(BLACK_LIST) | set(custom_black_list or ())) - set(custom_white_list or ())
        self.black_varnames = set(custom_black_varnames or ())
        self.dtype = dtype


CustomOpLists = AutoMixedPrecisionLists


def decorate(optimizer, amp_lists=None, init_loss_scaling=2 ** 15, incr_every_n_steps=1000,
             decr_every_n_nan_or_inf=2, incr_ratio=2.0, decr_ratio=0.8, use_dynamic_loss_scaling=True,
             use_pure_fp16=False, use_fp16_guard=None, use_bf16=False, use_promote=False, **kw):
    """Returns the optimizer; loss scaling is handled by GradScaler in our executor."""
    optimizer._amp_dtype = "bfloat16" if use_bf16 else "float16"
    optimizer._amp_level = "O2" if use_pure_fp16 else "O1"
    return optimizer


@contextlib.contextmanager
def fp16_guard():
    with auto_cast(True, level="O1", dtype="float16"):
        yield


class bf16:
    @staticmethod
    @contextlib.contextmanager
    def bf16_guard():
        with auto_cast(True, level="O1", dtype="bfloat16"):
            yield

    AutoMixedPrecisionListsBF16 = AutoMixedPrecisionLists

    @staticmethod
    def decorate_bf16(optimizer, amp_lists=None, use_pure_bf16=False, **kw):
        return decorate(optimizer, amp_lists, use_bf16=True, use_pure_fp16=use_pure_bf16)

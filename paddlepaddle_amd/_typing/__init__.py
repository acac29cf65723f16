"""paddle._typing: type aliases used in annotations. Reference: python/paddle/_typing/ (basic, dtype_like,
device_like, layout, shape)."""
from __future__ import annotations

from typing import Any, List, Sequence, Tuple, Union

import numpy as np

from ..framework.tensor import Tensor

EllipsisType = type(Ellipsis)
Numeric = Union[int, float, complex, np.number, Tensor]
NumericSequence = Sequence[Numeric]
NestedSequence = Union[Any, Sequence[Any]]
NestedList = Union[Any, List[Any]]
NestedNumericSequence = NestedSequence
NestedStructure = Any
TensorLike = Union[np.ndarray, Tensor, Numeric]
TensorOrTensors = Union[Tensor, Sequence[Tensor]]
TensorIndex = Any
ParamAttrLike = Any
DTypeLike = Union[str, np.dtype, type, Any]
PlaceLike = Union[str, Any]
DataLayout0D = str
DataLayout1D = str
DataLayout2D = str
DataLayout3D = str
DataLayoutND = str
DataLayoutImage = str
ShapeLike = Union[Sequence[int], Tuple[int, ...], Tensor]
Size1 = Union[int, Tuple[int]]
Size2 = Union[int, Tuple[int, int]]
Size3 = Union[int, Tuple[int, int, int]]
Size4 = Union[int, Tuple[int, int, int, int]]
Size5 = Union[int, Tuple[int, int, int, int, int]]
Size6 = Union[int, Tuple[int, int, int, int, int, int]]
SizeN = Sequence[int]

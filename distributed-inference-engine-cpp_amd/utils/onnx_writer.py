"""Pure-Python ONNX ModelProto writer (protobuf wire format, no `onnx` package needed).

The reference serves `models/resnet50-v2-7.onnx` (missing from the mount, `.MISSING_LARGE_BLOBS:1`);
neither `onnx` nor `protoc` is installed here, so the generators in `models/` emit the protobuf
bytes directly.  Field numbers follow onnx.proto (ModelProto/GraphProto/NodeProto/TensorProto/
AttributeProto/ValueInfoProto); the C++ reader is `csrc/onnx/onnx_model.cpp`.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Union

import numpy as np

FLOAT, UINT8, INT8, INT32, INT64, BOOL, FLOAT16, DOUBLE, BFLOAT16 = 1, 2, 3, 6, 7, 9, 10, 11, 16
_NP2ONNX = {
    np.dtype(np.float32): FLOAT,
    np.dtype(np.uint8): UINT8,
    np.dtype(np.int8): INT8,
    np.dtype(np.int32): INT32,
    np.dtype(np.int64): INT64,
    np.dtype(np.bool_): BOOL,
    np.dtype(np.float16): FLOAT16,
    np.dtype(np.float64): DOUBLE,
}


def _varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field_no: int, wire_type: int) -> bytes:
    return _varint((field_no << 3) | wire_type)


def f_varint(field_no: int, v: int) -> bytes:
    return _key(field_no, 0) + _varint(int(v))


def f_bytes(field_no: int, b: Union[bytes, bytearray]) -> bytes:
    return _key(field_no, 2) + _varint(len(b)) + bytes(b)


def f_str(field_no: int, s: str) -> bytes:
    return f_bytes(field_no, s.encode("utf-8"))


def f_float(field_no: int, v: float) -> bytes:
    return _key(field_no, 5) + struct.pack("<f", float(v))


def f_packed_varints(field_no: int, vals: Iterable[int]) -> bytes:
    payload = b"".join(_varint(int(v)) for v in vals)
    return f_bytes(field_no, payload)


def f_packed_floats(field_no: int, vals: Iterable[float]) -> bytes:
    vals = list(vals)
    return f_bytes(field_no, struct.pack("<%df" % len(vals), *vals))


# ---- messages -------------------------------------------------------------------------------------

def tensor_proto(name: str, arr: np.ndarray, use_raw: bool = True) -> bytes:
    arr = np.asarray(arr, order="C")  # (ascontiguousarray would turn a 0-d scalar into shape (1,))
    dt = _NP2ONNX[arr.dtype]
    out = bytearray()
    for d in arr.shape:
        out += f_varint(1, d)
    out += f_varint(2, dt)
    out += f_str(8, name)
    if use_raw:
        out += f_bytes(9, arr.astype(arr.dtype.newbyteorder("<"), copy=False).tobytes())
    elif dt == FLOAT:
        out += f_packed_floats(4, arr.reshape(-1).tolist())
    elif dt == INT64:
        out += f_packed_varints(7, arr.reshape(-1).tolist())
    elif dt in (INT32, UINT8, INT8, BOOL):
        out += f_packed_varints(5, arr.reshape(-1).astype(np.int64).tolist())
    else:
        raise ValueError("non-raw encoding unsupported for %s" % arr.dtype)
    return bytes(out)


def attribute_proto(name: str, value) -> bytes:
    out = bytearray(f_str(1, name))
    if isinstance(value, bool):
        value = int(value)
    if isinstance(value, int):
        out += f_varint(3, value) + f_varint(20, 2)
    elif isinstance(value, float):
        out += f_float(2, value) + f_varint(20, 1)
    elif isinstance(value, str):
        out += f_str(4, value) + f_varint(20, 3)
    elif isinstance(value, np.ndarray):
        out += f_bytes(5, tensor_proto(name, value)) + f_varint(20, 4)
    elif isinstance(value, (list, tuple)):
        if all(isinstance(v, (int, np.integer)) for v in value):
            out += f_packed_varints(8, value) + f_varint(20, 7)
        elif all(isinstance(v, (float, int)) for v in value):
            out += f_packed_floats(7, value) + f_varint(20, 6)
        else:
            for v in value:
                out += f_str(9, v)
            out += f_varint(20, 8)
    else:
        raise TypeError("unsupported attribute %s=%r" % (name, value))
    return bytes(out)


def node_proto(op_type: str, inputs: Sequence[str], outputs: Sequence[str], name: str = "", domain: str = "",
               **attrs) -> bytes:
    out = bytearray()
    for i in inputs:
        out += f_str(1, i)
    for o in outputs:
        out += f_str(2, o)
    if name:
        out += f_str(3, name)
    out += f_str(4, op_type)
    for k in sorted(attrs):
        out += f_bytes(5, attribute_proto(k, attrs[k]))
    if domain:
        out += f_str(7, domain)
    return bytes(out)


def value_info_proto(name: str, elem_type: int, dims: Sequence[Union[int, str]]) -> bytes:
    shape = bytearray()
    for d in dims:
        if isinstance(d, str):
            shape += f_bytes(1, f_str(2, d))
        else:
            shape += f_bytes(1, f_varint(1, d))
    tensor_type = f_varint(1, elem_type) + f_bytes(2, bytes(shape))
    type_proto = f_bytes(1, tensor_type)
    return f_str(1, name) + f_bytes(2, type_proto)


@dataclass
class GraphBuilder:
    """Accumulates nodes/initializers and serialises a ModelProto."""

    name: str = "graph"
    nodes: List[bytes] = field(default_factory=list)
    initializers: Dict[str, np.ndarray] = field(default_factory=dict)
    inputs: List[bytes] = field(default_factory=list)
    outputs: List[bytes] = field(default_factory=list)
    _counter: int = 0
    initializers_as_inputs: bool = False  # IR v3 style (gluoncv exports list weights as inputs)

    def fresh(self, prefix: str) -> str:
        self._counter += 1
        return "%s_%d" % (prefix, self._counter)

    def init(self, name: str, arr: np.ndarray) -> str:
        assert name not in self.initializers, name
        self.initializers[name] = np.asarray(arr, order="C")
        return name

    def const(self, arr, prefix: str = "const") -> str:
        return self.init(self.fresh(prefix), np.asarray(arr))

    def node(self, op: str, inputs: Sequence[str], outputs: Optional[Sequence[str]] = None, name: str = "",
             n_out: int = 1, **attrs) -> Union[str, List[str]]:
        if outputs is None:
            base = name or self.fresh(op.lower())
            outputs = [base if n_out == 1 else "%s_out%d" % (base, i) for i in range(n_out)]
        self.nodes.append(node_proto(op, inputs, outputs, name=name or outputs[0], **attrs))
        return outputs[0] if len(outputs) == 1 else list(outputs)

    def input(self, name: str, dims, elem_type: int = FLOAT) -> str:
        self.inputs.append(value_info_proto(name, elem_type, dims))
        return name

    def output(self, name: str, dims, elem_type: int = FLOAT) -> str:
        self.outputs.append(value_info_proto(name, elem_type, dims))
        return name

    def graph_proto(self) -> bytes:
        out = bytearray()
        for n in self.nodes:
            out += f_bytes(1, n)
        out += f_str(2, self.name)
        for k, v in self.initializers.items():
            out += f_bytes(5, tensor_proto(k, v))
        ins = list(self.inputs)
        if self.initializers_as_inputs:
            for k, v in self.initializers.items():
                ins.append(value_info_proto(k, _NP2ONNX[v.dtype], list(v.shape)))
        for i in ins:
            out += f_bytes(11, i)
        for o in self.outputs:
            out += f_bytes(12, o)
        return bytes(out)

    def model_proto(self, opset: int, ir_version: int = 8, producer: str = "die_amd") -> bytes:
        out = bytearray()
        out += f_varint(1, ir_version)
        out += f_str(2, producer)
        out += f_str(3, "0.1")
        out += f_bytes(7, self.graph_proto())
        out += f_bytes(8, f_str(1, "") + f_varint(2, opset))
        return bytes(out)

    def save(self, path: str, opset: int, ir_version: int = 8) -> None:
        with open(path, "wb") as f:
            f.write(self.model_proto(opset, ir_version))

"""TEST INFRASTRUCTURE: a minimal GGUF v3 writer (the public GGUF layout: "GGUF", u32 version,
u64 n_tensors, u64 n_kv, key/value pairs, tensor infos, data aligned to general.alignment).

The `gguf` package is absent from this image and no real model files exist here, so
the tests write their own files: synthetic Gemma models from the oracle's tensors, with the metadata
keys src/gemma_model.cpp:403-415 and :200-214 read.  Tensor shapes are given in ggml order
(ne[0] = row length)."""
import struct

import numpy as np

U8, I8, U16, I16, U32, I32, F32, BOOL, STR, ARR, U64, I64, F64 = range(13)
_SCALAR = {U8: "<B", I8: "<b", U16: "<H", I16: "<h", U32: "<I", I32: "<i", F32: "<f", BOOL: "<?",
           U64: "<Q", I64: "<q", F64: "<d"}
_NP = {U8: np.uint8, I8: np.int8, U16: np.uint16, I16: np.int16, U32: np.uint32, I32: np.int32,
       F32: np.float32, BOOL: np.uint8, U64: np.uint64, I64: np.int64, F64: np.float64}

# ggml type ids and (bytes per block, values per block)
GGML_BLOCK = {0: (4, 1), 1: (2, 1), 2: (18, 32), 8: (34, 32), 12: (144, 256), 14: (210, 256), 26: (4, 1)}


def _str(s):
    b = s.encode("utf-8") if isinstance(s, str) else bytes(s)
    return struct.pack("<Q", len(b)) + b


def tensor_nbytes(ggml_type, ne):
    bs, bl = GGML_BLOCK[ggml_type]
    n = bs * (ne[0] // bl)
    for d in ne[1:]:
        n *= d
    return n


class GGUFWriter:
    def __init__(self, alignment=32, version=3):
        self.kv = []        # (key, type, value, arr_type)
        self.tensors = []   # (name, ggml_type, ne, bytes)
        self.alignment = alignment
        self.version = version
        if alignment != 32:
            self.add("general.alignment", U32, alignment)

    def add(self, key, vtype, value, arr_type=None):
        self.kv.append((key, vtype, value, arr_type))

    def add_tensor(self, name, ggml_type, ne, data):
        data = bytes(np.ascontiguousarray(data).view(np.uint8).ravel()) if not isinstance(data, bytes) else data
        assert len(data) == tensor_nbytes(ggml_type, ne), (name, len(data), tensor_nbytes(ggml_type, ne))
        self.tensors.append((name, ggml_type, list(ne), data))

    def _value(self, vtype, value, arr_type):
        if vtype == STR:
            return _str(value)
        if vtype == ARR:
            out = struct.pack("<IQ", arr_type, len(value))
            if arr_type == STR:
                return out + b"".join(_str(v) for v in value)
            return out + np.asarray(value, dtype=_NP[arr_type]).tobytes()
        return struct.pack(_SCALAR[vtype], value)

    def to_bytes(self, offsets=None):
        head = struct.pack("<4sIQQ", b"GGUF", self.version, len(self.tensors), len(self.kv))
        for key, vtype, value, arr_type in self.kv:
            head += _str(key) + struct.pack("<I", vtype) + self._value(vtype, value, arr_type)
        a = self.alignment
        offs, off = [], 0
        for _, _, _, data in self.tensors:
            offs.append(off)
            off += (len(data) + a - 1) // a * a
        if offsets is not None:
            offs = offsets
        for (name, t, ne, _), o in zip(self.tensors, offs):
            head += _str(name) + struct.pack("<I", len(ne)) + struct.pack(f"<{len(ne)}Q", *ne) + struct.pack("<IQ", t, o)
        pad = (len(head) + a - 1) // a * a - len(head)
        body = bytearray()
        for (_, _, _, data), o in zip(self.tensors, offs):
            if o > (1 << 32):  # a deliberately bogus offset (malformed-file tests): header only
                continue
            if len(body) < o:
                body += b"\0" * (o - len(body))
            body[o:o + len(data)] = data
        tail = (len(body) + a - 1) // a * a - len(body)
        return head + b"\0" * pad + bytes(body) + b"\0" * tail

    def write(self, path, **kw):
        with open(path, "wb") as f:
            f.write(self.to_bytes(**kw))

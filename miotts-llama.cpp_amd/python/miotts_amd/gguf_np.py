"""Small read-only GGUF v2/v3 parser (numpy, memory-mapped) for harness code.

Reads KV metadata and tensor descriptors; tensor data is returned as raw bytes or,
for F32/F16/I32, as numpy arrays in ggml order reversed (numpy shape = ne[::-1]).
Nothing in the file is executed (no pickle).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Any, Dict, List

import numpy as np

_SCALAR = {0: "<B", 1: "<b", 2: "<H", 3: "<h", 4: "<I", 5: "<i", 6: "<f", 7: "<?",
           10: "<Q", 11: "<q", 12: "<d"}
_TYPE_BLOCK = {0: (1, 4), 1: (1, 2), 30: (1, 2), 24: (1, 1), 25: (1, 2), 26: (1, 4),
               2: (32, 18), 6: (32, 22), 8: (32, 34), 12: (256, 144), 14: (256, 210), 15: (256, 292)}


@dataclass
class Tensor:
    name: str
    ne: List[int]
    type: int
    offset: int
    reader: "GGUFReader" = field(repr=False)

    @property
    def nbytes(self) -> int:
        be, bb = _TYPE_BLOCK[self.type]
        n = int(np.prod(self.ne))
        return n // be * bb

    def raw(self) -> np.ndarray:
        start = self.reader.data_offset + self.offset
        return self.reader.mm[start:start + self.nbytes]

    def array(self) -> np.ndarray:
        dt = {0: np.float32, 1: np.float16, 26: np.int32, 24: np.int8, 25: np.int16}[self.type]
        return self.raw().view(dt).reshape(self.ne[::-1])


class GGUFReader:
    def __init__(self, path: str):
        self.mm = np.memmap(path, dtype=np.uint8, mode="r")
        b = self.mm
        self.pos = 0
        magic, ver = struct.unpack_from("<II", b, 0)
        if magic != 0x46554747 or ver not in (2, 3):
            raise ValueError(f"{path}: not GGUF v2/v3")
        n_t, n_kv = struct.unpack_from("<QQ", b, 8)
        self.pos = 24
        self.kv: Dict[str, Any] = {}
        self.kv_raw: List[tuple] = []  # (key, raw bytes of the typed value) in file order
        for _ in range(n_kv):
            k = self._str()
            p0 = self.pos
            t = self._u32()
            self.kv[k] = self._val(t)
            self.kv_raw.append((k, bytes(self.mm[p0:self.pos])))
        self.tensors: List[Tensor] = []
        for _ in range(n_t):
            name = self._str()
            nd = self._u32()
            ne = [self._u64() for _ in range(nd)]
            ty = self._u32()
            off = self._u64()
            self.tensors.append(Tensor(name, ne, ty, off, self))
        align = int(self.kv.get("general.alignment", 32))
        self.data_offset = (self.pos + align - 1) // align * align
        self.by_name = {t.name: t for t in self.tensors}

    def _u32(self) -> int:
        v = struct.unpack_from("<I", self.mm, self.pos)[0]
        self.pos += 4
        return v

    def _u64(self) -> int:
        v = struct.unpack_from("<Q", self.mm, self.pos)[0]
        self.pos += 8
        return v

    def _str(self) -> str:
        n = self._u64()
        s = bytes(self.mm[self.pos:self.pos + n]).decode("utf-8", errors="replace")
        self.pos += n
        return s

    def _val(self, t: int):
        if t == 8:
            return self._str()
        if t == 9:
            at = self._u32()
            n = self._u64()
            return [self._val(at) for _ in range(n)]
        fmt = _SCALAR[t]
        v = struct.unpack_from(fmt, self.mm, self.pos)[0]
        self.pos += struct.calcsize(fmt)
        return v

    def tensor(self, name: str) -> Tensor:
        return self.by_name[name]


def write_kv_gguf(path: str, kv: Dict[str, Any]) -> None:
    """Minimal GGUF v3 writer (metadata only, no tensors) for tokenizer tests.
    Values: str, bool, int (u32), float (f32), list[str], list[int] (i32), list[float] (f32),
    bytes (an array of u8, e.g. tokenizer.ggml.precompiled_charsmap)."""
    def s(x: str) -> bytes:
        b = x.encode("utf-8")
        return struct.pack("<Q", len(b)) + b

    out = bytearray(b"GGUF" + struct.pack("<IQQ", 3, 0, len(kv)))
    for k, v in kv.items():
        out += s(k)
        if isinstance(v, bool):
            out += struct.pack("<I?", 7, v)
        elif isinstance(v, int):
            out += struct.pack("<II", 4, v)
        elif isinstance(v, float):
            out += struct.pack("<If", 6, v)
        elif isinstance(v, str):
            out += struct.pack("<I", 8) + s(v)
        elif isinstance(v, (bytes, bytearray)):
            out += struct.pack("<IIQ", 9, 0, len(v)) + bytes(v)
        elif isinstance(v, list) and (not v or isinstance(v[0], str)):
            out += struct.pack("<IIQ", 9, 8, len(v)) + b"".join(s(x) for x in v)
        elif isinstance(v, list) and isinstance(v[0], float):
            out += struct.pack("<IIQ", 9, 6, len(v)) + b"".join(struct.pack("<f", x) for x in v)
        elif isinstance(v, list):
            out += struct.pack("<IIQ", 9, 5, len(v)) + b"".join(struct.pack("<i", x) for x in v)
        else:
            raise TypeError(k)
    with open(path, "wb") as f:
        f.write(bytes(out))


def _gguf_str(x: str) -> bytes:
    b = x.encode("utf-8")
    return struct.pack("<Q", len(b)) + b


def rewrite(src: str, dst: str, arch: str = None, extra_f32: str = None, drop_suffix: str = None) -> None:
    """Copy GGUF `src` to `dst` (loader tests): general.architecture replaced by `arch` when
    given, an extra 1-element F32 tensor named `extra_f32` appended when given, tensors whose
    name ends in `drop_suffix` left out when given."""
    r = GGUFReader(src)
    kvs = []
    for k, raw in r.kv_raw:
        if k == "general.architecture" and arch is not None:
            raw = struct.pack("<I", 8) + _gguf_str(arch)
        kvs.append(_gguf_str(k) + raw)
    tens = [(t.name, t.ne, t.type, t.raw()) for t in r.tensors
            if not (drop_suffix and t.name.endswith(drop_suffix))]
    if extra_f32:
        tens.append((extra_f32, [1], 0, np.zeros(4, np.uint8)))
    align = int(r.kv.get("general.alignment", 32))
    infos, off = [], 0
    for name, ne, ty, data in tens:
        infos.append(_gguf_str(name) + struct.pack("<I", len(ne)) + b"".join(struct.pack("<Q", n) for n in ne)
                     + struct.pack("<IQ", ty, off))
        off = (off + len(data) + align - 1) // align * align
    head = b"GGUF" + struct.pack("<IQQ", 3, len(tens), len(kvs)) + b"".join(kvs) + b"".join(infos)
    with open(dst, "wb") as f:
        f.write(head)
        f.write(b"\0" * ((len(head) + align - 1) // align * align - len(head)))
        for _, _, _, data in tens:
            b = bytes(data)
            f.write(b)
            f.write(b"\0" * ((len(b) + align - 1) // align * align - len(b)))

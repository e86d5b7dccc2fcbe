"""Value codecs: Python object -> the exact bytes Redisson would send.

The engine hashes whatever bytes arrive (PFADD elements, Bloom elements), so
the host side must reproduce Redisson's codec output byte for byte:

* ``JsonJacksonCodec`` (the default codec, M:Config.java:68-70) with the
  default typing of M:codec/JsonJacksonCodec.java:86-117: NON_FINAL types get
  class info, and ``java.lang.Long`` is forced typed (:103-106).  With
  ``As.PROPERTY`` on a scalar / array Jackson falls back to a wrapper array,
  so a Long encodes as ``["java.lang.Long",123]`` and an ``Object[]`` as
  ``["[Ljava.lang.Object;",[...]]``.  Natural JSON types (String, Integer,
  Boolean) stay untyped.  Byte forms are restated from Jackson 2.6.5
  behaviour (no JVM here): parity of the typed forms is UNPINNED until checked
  on a JVM (Oracle).
* ``StringCodec`` (``toString().getBytes(UTF-8)``), ``LongCodec``,
  ``ByteArrayCodec``.

Java boxing has no Python analogue: ``JLong(5)`` is a ``java.lang.Long``,
``JInteger(5)`` an ``Integer``; a bare Python ``int`` is an ``Integer`` when it
fits 32 bits (what a Java int literal autoboxes to) and a ``Long`` otherwise.
"""
from __future__ import annotations

import base64


class JLong(int):
    """A value that is a java.lang.Long on the Java side."""


class JInteger(int):
    """A value that is a java.lang.Integer on the Java side."""


_HEX = "0123456789ABCDEF"


def _json_string(s: str) -> str:
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif o < 32:
            short = {8: "b", 9: "t", 10: "n", 12: "f", 13: "r"}.get(o)
            out.append("\\" + short if short else "\\u00" + _HEX[o >> 4] + _HEX[o & 15])
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


class Codec:
    name = "codec"

    def encode(self, obj) -> bytes:  # value encoder
        raise NotImplementedError


class JsonJacksonCodec(Codec):
    name = "JsonJacksonCodec"

    def _value(self, obj, typed_context: bool) -> str:
        # typed_context: declared type is Object (element of Object[] / top level)
        if obj is None:
            return "null"
        if isinstance(obj, bool):
            return "true" if obj else "false"
        if isinstance(obj, JLong) or (isinstance(obj, int) and not isinstance(obj, JInteger)
                                      and not (-(1 << 31) <= obj < (1 << 31))):
            if not (-(1 << 63) <= obj < (1 << 63)):
                raise OverflowError("value does not fit a java.lang.Long")
            return '["java.lang.Long",%d]' % int(obj)
        if isinstance(obj, int):
            return "%d" % int(obj)
        if isinstance(obj, str):
            return _json_string(obj)
        if isinstance(obj, (bytes, bytearray)):
            return _json_string(base64.b64encode(bytes(obj)).decode("ascii"))
        if isinstance(obj, (list, tuple)):
            inner = ",".join(self._value(x, True) for x in obj)
            return '["[Ljava.lang.Object;",[%s]]' % inner
        raise TypeError(f"JsonJacksonCodec emulation does not cover {type(obj).__name__}")

    def encode(self, obj) -> bytes:
        return self._value(obj, True).encode("utf-8")


class StringCodec(Codec):
    name = "StringCodec"

    def encode(self, obj) -> bytes:
        if isinstance(obj, (bytes, bytearray)):
            return bytes(obj)
        return str(obj).encode("utf-8")


class LongCodec(StringCodec):
    name = "LongCodec"

    def encode(self, obj) -> bytes:
        return b"%d" % int(obj)


class ByteArrayCodec(Codec):
    name = "ByteArrayCodec"

    def encode(self, obj) -> bytes:
        return bytes(obj)


def params_bytes(param) -> bytes:
    """DefaultParamsEncoder: raw byte[] as-is, else toString().getBytes(UTF-8)."""
    if isinstance(param, (bytes, bytearray)):
        return bytes(param)
    return str(param).encode("utf-8")

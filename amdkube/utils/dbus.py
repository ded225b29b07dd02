"""A minimal D-Bus client: the wire protocol spoken to systemd for the systemd cgroup driver.

The reference drives systemd through godbus (vendor/github.com/godbus/dbus, used by
libcontainer/cgroups/systemd and go-systemd's StartTransientUnit). No D-Bus library ships in
this image, so this module speaks the protocol directly over the unix socket:
* SASL EXTERNAL authentication with the caller's uid, then BEGIN;
* little-endian messages — a 12-byte fixed header, the header-field array a(yv) padded to 8,
  then the body — with the alignment rules of the marshalling spec (y 1, n/q 2, b/i/u/s/o/a 4,
  x/t/d/(…)/{…} 8, g/v 1);
* `Hello` on a message bus (the system bus); none on systemd's private socket, which is
  peer-to-peer.
Values: basic types map to Python ints / str / bool / float; arrays to lists; structs and dict
entries to tuples; a variant is a `(signature, value)` pair. Signals and method calls that
arrive while a reply is awaited are dropped (nothing here subscribes to any).
"""
from __future__ import annotations

import os
import socket
import threading
import struct

METHOD_CALL, METHOD_RETURN, ERROR, SIGNAL = 1, 2, 3, 4
F_PATH, F_INTERFACE, F_MEMBER, F_ERROR_NAME, F_REPLY_SERIAL, F_DESTINATION, F_SENDER, F_SIGNATURE = range(1, 9)
_FIELD_SIG = {F_PATH: "o", F_INTERFACE: "s", F_MEMBER: "s", F_ERROR_NAME: "s", F_REPLY_SERIAL: "u",
              F_DESTINATION: "s", F_SENDER: "s", F_SIGNATURE: "g"}
_FIXED = {"y": ("B", 1), "b": ("I", 4), "n": ("h", 2), "q": ("H", 2), "i": ("i", 4), "u": ("I", 4),
          "x": ("q", 8), "t": ("Q", 8), "d": ("d", 8), "h": ("I", 4)}
_ALIGN = {"y": 1, "b": 4, "n": 2, "q": 2, "i": 4, "u": 4, "x": 8, "t": 8, "d": 8, "h": 4, "s": 4, "o": 4, "g": 1,
          "v": 1, "a": 4, "(": 8, "{": 8}


class DBusError(Exception):
    def __init__(self, name: str, message: str = ""):
        super().__init__(f"{name}: {message}" if message else name)
        self.name, self.message = name, message


def split_signature(sig: str) -> list[str]:
    """The complete types of a signature, in order."""
    out, i = [], 0
    while i < len(sig):
        j = _end_of(sig, i)
        out.append(sig[i:j])
        i = j
    return out


def _end_of(sig: str, i: int) -> int:
    c = sig[i]
    if c == "a":
        return _end_of(sig, i + 1)
    if c in "({":
        close = ")" if c == "(" else "}"
        j = i + 1
        while sig[j] != close:
            j = _end_of(sig, j)
        return j + 1
    if c in _ALIGN:
        return i + 1
    raise ValueError(f"bad signature {sig!r} at {i}")


class _Writer:
    def __init__(self):
        self.buf = bytearray()

    def pad(self, n: int):
        self.buf += b"\0" * (-len(self.buf) % n)

    def write(self, sig: str, v):
        c = sig[0]
        self.pad(_ALIGN[c])
        if c in _FIXED:
            fmt, _ = _FIXED[c]
            self.buf += struct.pack("<" + fmt, int(bool(v)) if c == "b" else v)
        elif c in "so":
            b = v.encode()
            self.buf += struct.pack("<I", len(b)) + b + b"\0"
        elif c == "g":
            b = v.encode()
            self.buf += struct.pack("<B", len(b)) + b + b"\0"
        elif c == "v":
            vsig, val = v
            self.write("g", vsig)
            self.write(vsig, val)
        elif c == "a":
            elem = sig[1:]
            at = len(self.buf)
            self.buf += b"\0\0\0\0"
            self.pad(_ALIGN[elem[0]])                      # padding before the first element is not counted
            start = len(self.buf)
            items = v.items() if isinstance(v, dict) else v
            for x in items:
                self.write(elem, x)
            struct.pack_into("<I", self.buf, at, len(self.buf) - start)
        elif c in "({":
            for t, x in zip(split_signature(sig[1:-1]), v):
                self.write(t, x)
        else:
            raise ValueError(f"cannot marshal {sig!r}")


class _Reader:
    def __init__(self, data: bytes, pos: int = 0):
        self.data, self.pos = data, pos

    def align(self, n: int):
        self.pos += -self.pos % n

    def read(self, sig: str):
        c = sig[0]
        self.align(_ALIGN[c])
        if c in _FIXED:
            fmt, size = _FIXED[c]
            (v,) = struct.unpack_from("<" + fmt, self.data, self.pos)
            self.pos += size
            return bool(v) if c == "b" else v
        if c in "so":
            (n,) = struct.unpack_from("<I", self.data, self.pos)
            s = self.data[self.pos + 4:self.pos + 4 + n].decode()
            self.pos += 4 + n + 1
            return s
        if c == "g":
            n = self.data[self.pos]
            s = self.data[self.pos + 1:self.pos + 1 + n].decode()
            self.pos += 1 + n + 1
            return s
        if c == "v":
            vsig = self.read("g")
            return vsig, self.read(vsig)
        if c == "a":
            (n,) = struct.unpack_from("<I", self.data, self.pos)
            self.pos += 4
            elem = sig[1:]
            self.align(_ALIGN[elem[0]])
            end, out = self.pos + n, []
            while self.pos < end:
                out.append(self.read(elem))
            return dict(out) if elem[0] == "{" else out
        if c in "({":
            return tuple(self.read(t) for t in split_signature(sig[1:-1]))
        raise ValueError(f"cannot unmarshal {sig!r}")


def marshal_body(sig: str, args) -> bytes:
    w = _Writer()
    for t, a in zip(split_signature(sig), args):
        w.write(t, a)
    return bytes(w.buf)


def unmarshal_body(sig: str, data: bytes) -> list:
    r = _Reader(data)
    return [r.read(t) for t in split_signature(sig)]


def encode_message(mtype: int, serial: int, fields: dict, sig: str = "", args=(), flags: int = 0) -> bytes:
    body = marshal_body(sig, args) if sig else b""
    if sig:
        fields = {**fields, F_SIGNATURE: sig}
    w = _Writer()
    w.buf += struct.pack("<cBBBII", b"l", mtype, flags, 1, len(body), serial)
    w.write("a(yv)", [(code, (_FIELD_SIG[code], val)) for code, val in sorted(fields.items())])
    w.pad(8)
    return bytes(w.buf) + body


def decode_message(data: bytes):
    """One complete message -> (type, flags, serial, fields, body values)."""
    if data[:1] != b"l":
        raise DBusError("org.freedesktop.DBus.Error.InvalidArgs", "big-endian messages are not supported")
    mtype, flags, _version, blen, serial = struct.unpack_from("<BBBII", data, 1)
    r = _Reader(data, 12)
    fields = {code: val for code, (_s, val) in r.read("a(yv)")}
    r.align(8)
    body = data[r.pos:r.pos + blen]
    sig = fields.get(F_SIGNATURE, "")
    return mtype, flags, serial, fields, (unmarshal_body(sig, body) if sig else [])


def message_length(head: bytes) -> int:
    """Total length of the message whose first 16 bytes are `head`."""
    _e, _t, _f, _v, blen, _s, flen = struct.unpack_from("<cBBBIII", head, 0)
    hdr = 16 + flen
    return hdr + (-hdr % 8) + blen


class Connection:
    """A blocking connection to a bus (or to a peer such as systemd's private socket)."""

    def __init__(self, path: str, bus: bool = True, timeout: float = 10.0):
        self.path, self.bus, self.timeout = path, bus, timeout
        self.sock: socket.socket | None = None
        self.serial = 0
        self.unique_name = ""
        self._buf = b""
        # one caller at a time: a call sends, then reads until its own reply; two threads
        # interleaving would each discard the other's reply (and share _buf)
        self._lock = threading.RLock()

    def connect(self) -> "Connection":
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.settimeout(self.timeout)
        s.connect(self.path)
        self.sock = s
        s.sendall(b"\0AUTH EXTERNAL " + str(os.getuid()).encode().hex().encode() + b"\r\n")
        line = self._readline()
        if not line.startswith(b"OK"):
            self.close()
            raise DBusError("org.freedesktop.DBus.Error.AuthFailed", line.decode(errors="replace"))
        s.sendall(b"BEGIN\r\n")
        if self.bus:
            (self.unique_name,) = self.call("org.freedesktop.DBus", "/org/freedesktop/DBus", "org.freedesktop.DBus", "Hello")
        return self

    def close(self):
        if self.sock is not None:
            self.sock.close()
            self.sock = None

    def _readline(self) -> bytes:
        while b"\r\n" not in self._buf:
            chunk = self.sock.recv(4096)
            if not chunk:
                raise DBusError("org.freedesktop.DBus.Error.Disconnected", "connection closed during authentication")
            self._buf += chunk
        line, _, self._buf = self._buf.partition(b"\r\n")
        return line

    def _recv_exact(self, n: int) -> bytes:
        while len(self._buf) < n:
            chunk = self.sock.recv(max(4096, n - len(self._buf)))
            if not chunk:
                raise DBusError("org.freedesktop.DBus.Error.Disconnected", "connection closed")
            self._buf += chunk
        out, self._buf = self._buf[:n], self._buf[n:]
        return out

    def _read_message(self):
        head = self._recv_exact(16)
        rest = self._recv_exact(message_length(head) - 16)
        return decode_message(head + rest)

    def call(self, destination: str | None, path: str, interface: str, member: str, sig: str = "", *args):
        """A method call; returns the reply's body values or raises DBusError."""
        with self._lock:
            if self.sock is None:
                raise DBusError("org.freedesktop.DBus.Error.Disconnected", "not connected")
            self.serial += 1
            serial = self.serial
            fields = {F_PATH: path, F_INTERFACE: interface, F_MEMBER: member}
            if destination:
                fields[F_DESTINATION] = destination
            self.sock.sendall(encode_message(METHOD_CALL, serial, fields, sig, args))
            while True:
                mtype, _flags, _s, f, body = self._read_message()
                if f.get(F_REPLY_SERIAL) != serial:
                    continue                      # a signal
                if mtype == ERROR:
                    raise DBusError(f.get(F_ERROR_NAME, "org.freedesktop.DBus.Error.Failed"),
                                    body[0] if body and isinstance(body[0], str) else "")
                return body

"""Python side of the minimal erl_nif runtime (tests/nif_rt/erl_nif_rt.c) --
TEST INFRASTRUCTURE ONLY.

Python values <-> the runtime's external format, and calls of the NIF's
functions (nif/antidote_gpu_nif.c, linked into libagn_nif_rt.so):
  int <-> integer, Atom <-> atom (True / False <-> true / false), tuple <->
  tuple, list <-> proper list, bytes <-> binary, Res <-> resource.
A call that raises comes back as NifBadarg / NifRaise (the exception's
reason decoded)."""
import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libagn_nif_rt.so")


class Atom(str):
    def __repr__(self):
        return f"Atom({str.__repr__(self)})"


class Res:
    """A resource term (opaque pointer)."""

    def __init__(self, ptr):
        self.ptr = ptr

    def __repr__(self):
        return f"Res({self.ptr:#x})"


class NifBadarg(Exception):
    pass


class NifRaise(Exception):
    def __init__(self, reason):
        super().__init__(reason)
        self.reason = reason


def encode(v, out=None):
    out = bytearray() if out is None else out
    if isinstance(v, bool):
        v = Atom("true" if v else "false")
    if isinstance(v, Atom):
        b = str(v).encode()
        out += b"A" + len(b).to_bytes(4, "little") + b
    elif isinstance(v, int):
        out += b"I" + v.to_bytes(16, "little", signed=True)
    elif isinstance(v, tuple):
        out += b"T" + len(v).to_bytes(4, "little")
        for x in v:
            encode(x, out)
    elif isinstance(v, list):
        for x in v:
            out += b"L"
            encode(x, out)
        out += b"N"
    elif isinstance(v, (bytes, bytearray)):
        out += b"B" + len(v).to_bytes(4, "little") + bytes(v)
    elif isinstance(v, Res):
        out += b"R" + v.ptr.to_bytes(8, "little")
    else:
        raise TypeError(f"no term for {v!r}")
    return out


def decode(b):
    v, i = _dec(b, 0)
    assert i == len(b), (i, len(b))
    return v


def _dec(b, i):
    t = b[i:i + 1]
    i += 1
    if t == b"I":
        return int.from_bytes(b[i:i + 16], "little", signed=True), i + 16
    if t in (b"A", b"B"):
        n = int.from_bytes(b[i:i + 4], "little")
        s = bytes(b[i + 4:i + 4 + n])
        return (Atom(s.decode()) if t == b"A" else s), i + 4 + n
    if t == b"N":
        return [], i
    if t == b"R":
        return Res(int.from_bytes(b[i:i + 8], "little")), i + 8
    if t == b"T":
        n = int.from_bytes(b[i:i + 4], "little")
        i += 4
        out = []
        for _ in range(n):
            x, i = _dec(b, i)
            out.append(x)
        return tuple(out), i
    if t == b"L":
        out = []
        i -= 1
        while b[i:i + 1] == b"L":
            x, i = _dec(b, i + 1)
            out.append(x)
        tail, i = _dec(b, i)
        assert tail == [], "improper list"
        return out, i
    raise ValueError(f"bad tag {t!r} at {i - 1}")


def build(force=False):
    """make -C tests/nif_rt (gcc; links antidote_amd/libantidote_gpu.so)."""
    subprocess.check_call(["make", "-s", "-C", HERE] + (["-B"] if force else []))
    return LIB


class NifRuntime:
    """The NIF module loaded through the runtime; call(name, *args)."""

    def __init__(self):
        if not os.path.exists(LIB):
            build()
        self.lib = lib = C.CDLL(LIB)
        P = C.c_void_p
        lib.rt_load.restype = C.c_int
        lib.rt_env_new.restype = P
        lib.rt_env_free.argtypes = [P]
        lib.rt_decode.restype = C.c_uint64
        lib.rt_decode.argtypes = [P, C.c_char_p, C.c_size_t]
        lib.rt_encode.restype = C.c_long
        lib.rt_encode.argtypes = [C.c_uint64, C.POINTER(P)]
        lib.rt_free_buf.argtypes = [P]
        lib.rt_call.restype = C.c_uint64
        lib.rt_call.argtypes = [P, C.c_char_p, C.c_int, C.POINTER(C.c_uint64),
                                C.POINTER(C.c_int)]
        lib.rt_exc_reason.restype = C.c_uint64
        lib.rt_exc_reason.argtypes = [P]
        lib.rt_keep.restype = C.c_uint64
        lib.rt_keep.argtypes = [C.c_uint64]
        lib.rt_release.argtypes = [C.c_uint64]
        lib.rt_live_resources.restype = C.c_long
        assert lib.rt_load() == 0, "NIF load callback failed"
        self.kept = []

    def _out(self, t):
        buf = C.c_void_p()
        n = self.lib.rt_encode(t, C.byref(buf))
        assert n >= 0, "unencodable term"
        try:
            return decode(C.string_at(buf, n))
        finally:
            self.lib.rt_free_buf(buf)

    def call(self, name, *args, keep=False):
        """Name(Args...) -> the decoded result; keep=True: hold a reference on
        each resource in the result (the result outlives this call's env)."""
        env = self.lib.rt_env_new()
        try:
            argv = (C.c_uint64 * max(len(args), 1))()
            for i, a in enumerate(args):
                b = bytes(encode(a))
                argv[i] = self.lib.rt_decode(env, b, len(b))
                assert argv[i], f"argument {i} did not decode"
            exc = C.c_int()
            r = self.lib.rt_call(env, name.encode(), len(args), argv, C.byref(exc))
            if exc.value == -1:
                raise AttributeError(f"no NIF {name}/{len(args)}")
            if exc.value == 1:
                raise NifBadarg(name)
            if exc.value == 2:
                raise NifRaise(self._out(self.lib.rt_exc_reason(env)))
            out = self._out(r)
            if keep:
                self._keep(out)
            return out
        finally:
            self.lib.rt_env_free(env)

    def _keep(self, v):
        if isinstance(v, Res):
            env = self.lib.rt_env_new()
            b = bytes(encode(v))
            t = self.lib.rt_decode(env, b, len(b))
            self.kept.append(self.lib.rt_keep(t))
            self.lib.rt_env_free(env)
        elif isinstance(v, (tuple, list)):
            for x in v:
                self._keep(x)

    def release_all(self):
        """Drop the references keep=True took (destructors run)."""
        while self.kept:
            self.lib.rt_release(self.kept.pop())

    def live_resources(self):
        return self.lib.rt_live_resources()


def roundtrip(rt, v):
    """v through the C runtime: decoded into a term, encoded back."""
    env = rt.lib.rt_env_new()
    try:
        b = bytes(encode(v))
        t = rt.lib.rt_decode(env, b, len(b))
        assert t, "did not decode"
        return rt._out(t)
    finally:
        rt.lib.rt_env_free(env)

"""ctypes binding of the native CLI (kafkabalancer_amd/host, kb_cli_run): the
reference's run(stdin, stdout, stderr, args) (kafkabalancer.go:72)."""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libkbhost.so")
BIN_PATH = os.path.join(_HERE, "lib", "kafkabalancer")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libkbhost.so not built; run __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        L.kb_cli_run.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.c_char_p, C.c_size_t, C.c_int,
                                 C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                 C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
        L.kb_cli_run.restype = C.c_int
        L.kb_cli_free.argtypes = [C.c_void_p]
        L.kb_codec_roundtrip.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.POINTER(C.c_void_p),
                                         C.POINTER(C.c_size_t), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                         C.POINTER(C.c_int64)]
        L.kb_codec_roundtrip.restype = C.c_int
        _lib = L
    return _lib


def run(args, stdin=None, fail_output=False):
    """Returns (exit_code, stdout_bytes, stderr_text).  stdin=None means no reader."""
    argv = (C.c_char_p * len(args))(*[a.encode() for a in args])
    out, err = C.c_void_p(), C.c_void_p()
    olen, elen = C.c_size_t(), C.c_size_t()
    data = stdin if stdin is None or isinstance(stdin, bytes) else stdin.encode()
    rc = lib().kb_cli_run(len(args), argv, data, len(data) if data else 0, int(fail_output),
                          C.byref(out), C.byref(olen), C.byref(err), C.byref(elen))
    o = C.string_at(out.value, olen.value) if out.value else b""
    e = C.string_at(err.value, elen.value).decode(errors="replace") if err.value else ""
    lib().kb_cli_free(out)
    lib().kb_cli_free(err)
    return rc, o, e


CODEC_DEFAULT, CODEC_DOM, CODEC_FAST = 0, 1, 2


def codec_roundtrip(data, mode=CODEC_DEFAULT):
    """Decode JSON `data` like GetPartitionListFromReader and encode it again like
    WritePartitionList (codecs.go:15-27, 84-93).  Returns (rc, bytes, t_parse_s,
    t_encode_s, n_partitions): rc 0 = encoded bytes, 1 = the error text, 2 = the
    one-pass decoder gave up (mode CODEC_FAST only)."""
    out = C.c_void_p()
    olen = C.c_size_t()
    tp, te = C.c_double(), C.c_double()
    n = C.c_int64()
    rc = lib().kb_codec_roundtrip(data, len(data), mode, C.byref(out), C.byref(olen), C.byref(tp), C.byref(te),
                                  C.byref(n))
    o = b""
    if out.value:
        o = C.string_at(out.value, olen.value)
        lib().kb_cli_free(out)
    return rc, o, tp.value, te.value, n.value

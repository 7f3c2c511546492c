"""ctypes wrapper of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker; never by the product (libbert.so).
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "_build", "liboracle.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle not built: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_load.restype = ctypes.c_void_p
        L.oracle_load.argtypes = [ctypes.c_char_p]
        L.oracle_free.argtypes = [ctypes.c_void_p]
        L.oracle_hparams.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32)]
        L.oracle_id_to_token.restype = ctypes.c_char_p
        L.oracle_id_to_token.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        L.oracle_tokenize.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int32),
                                      ctypes.POINTER(ctypes.c_int32), ctypes.c_int32, ctypes.c_int32]
        for fn in (L.oracle_forward_batch, L.oracle_forward_fake_batch):
            fn.restype = ctypes.c_int
            fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int32),
                           ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_float)]
        L.oracle_encode_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_float),
                                          ctypes.POINTER(ctypes.c_int32)]
        L.oracle_quantize_file.restype = ctypes.c_int
        L.oracle_quantize_file.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        L.oracle_f32_to_f16.restype = ctypes.c_uint16
        L.oracle_f32_to_f16.argtypes = [ctypes.c_float]
        L.oracle_f16_to_f32.restype = ctypes.c_float
        L.oracle_f16_to_f32.argtypes = [ctypes.c_uint16]
        L.oracle_gelu.restype = ctypes.c_float
        L.oracle_gelu.argtypes = [ctypes.c_float]
        L.oracle_exp.restype = ctypes.c_float
        L.oracle_exp.argtypes = [ctypes.c_float]
        L.oracle_quantize_row.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_dequantize_row.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        for fn in (L.oracle_forward_batch_ex, L.oracle_forward_fake_batch_ex):
            fn.restype = ctypes.c_int
            fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int32),
                           ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_float)]
        _lib = L
    return _lib


def _i32(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def _f32(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class Oracle:
    """One loaded model file (restatement of bert_load_from_file, bert.cpp:423-786)."""

    def __init__(self, path):
        self.h = lib().oracle_load(path.encode())
        if not self.h:
            raise RuntimeError("oracle failed to load " + path)
        hp = (ctypes.c_int32 * 7)()
        lib().oracle_hparams(self.h, hp)
        (self.n_vocab, self.n_max_tokens, self.n_embd, self.n_intermediate,
         self.n_head, self.n_layer, self.ftype) = list(hp)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_free(self.h)
            self.h = None

    def tokenize(self, text, n_max_tokens=None):
        if isinstance(text, str):
            text = text.encode("utf-8")
        n_max = self.n_max_tokens if n_max_tokens is None else n_max_tokens
        cap = n_max + len(text) + 8
        buf = np.zeros(cap, np.int32)
        n = ctypes.c_int32(0)
        lib().oracle_tokenize(self.h, text, _i32(buf), ctypes.byref(n), n_max, cap)
        return [int(x) for x in buf[: n.value]]

    def id_to_token(self, i):
        return lib().oracle_id_to_token(self.h, i)

    def _fwd(self, fn, ids_list, n_threads, activations="q8"):
        """activations "q8": the reference's arithmetic (q4/q8 weights x q8_0 / q8_1
        re-quantized activations); "f32": the diagnostic mode (the same weights x the
        f32 activations, a per-call argument of oracle_forward_batch_ex) -- only to
        measure how far the reference's activation rounding moves an embedding, never
        as the parity bar."""
        assert activations in ("q8", "f32")
        flat = np.ascontiguousarray(np.concatenate([np.asarray(x, np.int32) for x in ids_list]))
        lens = np.asarray([len(x) for x in ids_list], np.int32)
        out = np.zeros((len(ids_list), self.n_embd), np.float32)
        rc = fn(self.h, n_threads, 1 if activations == "f32" else 0, len(ids_list), _i32(flat), _i32(lens), _f32(out))
        if rc != 0:
            return None
        return out

    def forward_batch(self, ids_list, n_threads=8, activations="q8"):
        return self._fwd(lib().oracle_forward_batch_ex, ids_list, n_threads, activations)

    def forward_fake_batch(self, ids_list, n_threads=8, activations="q8"):
        return self._fwd(lib().oracle_forward_fake_batch_ex, ids_list, n_threads, activations)

    def encode_batch(self, texts, n_batch_size, n_threads=8):
        n = len(texts)
        arr = (ctypes.c_char_p * n)(*[t.encode("utf-8") if isinstance(t, str) else t for t in texts])
        out = np.zeros((n, self.n_embd), np.float32)
        written = np.zeros(n, np.int32)
        lib().oracle_encode_batch(self.h, n_threads, n_batch_size, n, arr, _f32(out), _i32(written))
        return out, written.astype(bool)


def quantize_file(src, dst, itype):
    return lib().oracle_quantize_file(src.encode(), dst.encode(), itype)


def f32_to_f16_bits(x):
    return int(lib().oracle_f32_to_f16(float(x)))

#!/usr/bin/env python3
"""Regenerates the committed golden fixtures under tests/golden/.

Runs ONLY in the build container (needs /root/reference and the oracle):
  1. tokenizer goldens: token ids from the reference's OWN tokenizer source
     (bert.cpp:195-417, compiled by oracle/build_ref.sh into oracle/_ref/libreftok.so)
     over the reference's prompt files + edge cases, with a synthetic vocab
     (no real vocab file exists offline).
  2. model fixtures: a tiny random BertModel saved locally, converted by the
     reference's own converter models/convert-to-ggml.py (f32 and f16 files).
  3. forward goldens: an independent torch/transformers BertModel forward with
     the reference's era constants (tanh GELU, LayerNorm eps 1e-5, masked mean
     pool, L2 norm) plus the oracle's own outputs on the same ids.
Nothing here is imported by the product or by the GPU tests.
"""
import ctypes
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("REF", "/root/reference")
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib  # noqa: E402


def build_vocab():
    v = ["[PAD]"] + ["[unused%d]" % i for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    assert v[100] == "[UNK]" and v[101] == "[CLS]" and v[102] == "[SEP]"
    punct = list("!\"#$%&'()*+,-./:;<=>?@[\\]^_`{|}~")
    chars = punct + list("0123456789") + [chr(c) for c in range(ord("a"), ord("z") + 1)]
    v += chars
    v += ["##" + c for c in "0123456789abcdefghijklmnopqrstuvwxyz"]
    # words from the reference's own sample texts
    words = {}
    with open(os.path.join(REF, "examples", "sample_client_texts.txt"), encoding="utf-8") as f:
        for line in f:
            for w in "".join(ch if ch.isalnum() else " " for ch in line.lower()).split():
                words[w] = words.get(w, 0) + 1
    top = [w for w, _ in sorted(words.items(), key=lambda kv: (-kv[1], kv[0])) if len(w) > 1][:400]
    v += top
    v += ["##" + s for s in ["s", "ing", "ed", "ly", "er", "tion", "al", "ment", "able", "ness", "ies", "re"]]
    v += ["hello", "world", "store", "buy", "apple", "banana", "welcome", "cloud", "outside", "anywhere",
          "stack", "calculate", "int", "char", "return", "push", "pop", "result", "express", "##ion",
          "evaluate", "##post", "##fix", "digit", "gpt", "accent", "umlaut"]
    # CJK / kana characters of the reference prompts (test_prompts.txt:4-8)
    with open(os.path.join(REF, "examples", "test_prompts.txt"), encoding="utf-8") as f:
        cjk = sorted({ch for ch in f.read() if ord(ch) > 0x2E80})
    v += cjk[: len(cjk) // 2]          # leave half unknown on purpose
    v += ["##" + c for c in cjk[:10]]
    # map-semantics edge cases: duplicates (first wins / last wins), odd entries
    v += ["the", "##s", "##", "#", "a##b", "café", "##é", "[UNK]"]
    return v


def edge_texts():
    t = [
        "", "   ", "hello", "Hello World", "HÉLLO wörld ÀÁÂÃÄÅ àáâãäå ÈÉÊË ÌÍÎÏ ÒÓÔÕÖ ÙÚÛÜ Ýý Çç Ññ Æ æ Ø",
        "x!x", "a...b", "don't stop", "I ❤️ 🍕 pizza", "tab\tsep\nnewline\r\nend\x0bvt\x0cff",
        "，。！、「」ＡＢＣ１２３", "中文English混合mixed", "ünïcödé naïve café",
        "unknownzzqq words qqq", "123456789 3.14159 1,000,000", "the the the", "##s", "a##b",
        "email@example.com http://x.y/z?q=1&r=2", "(parenthesis) [brackets] {braces} <angles>",
        " ".join(["the"] * 600), "a" * 600, "medicare " * 300, "你" * 300,
        "question? answer! statement. list: a; b, c",
    ]
    return [s.encode("utf-8") for s in t] + [b"\xff\xfe abc \xc3", b"abc\xe4\xbd", b"\xe4\xbd\xa0\xe5", b"\x80\x81 x"]


def reftok_ids(vocab, texts, n_max):
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libreftok.so"))
    lib.reftok_new.restype = ctypes.c_void_p
    lib.reftok_add.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int]
    lib.reftok_tokenize.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int32),
                                    ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]
    lib.reftok_free.argtypes = [ctypes.c_void_p]
    ctx = lib.reftok_new()
    for i, w in enumerate(vocab):
        b = w.encode("utf-8")
        lib.reftok_add(ctx, b, len(b), i)
    out = []
    for s in texts:
        buf = (ctypes.c_int32 * (n_max + 100000))()
        n = ctypes.c_int32(0)
        lib.reftok_tokenize(ctx, s, buf, ctypes.byref(n), n_max)
        out.append([int(x) for x in buf[: n.value]])
    lib.reftok_free(ctx)
    return out


def make_tokenizer_golden(vocab):
    with open(os.path.join(REF, "examples", "test_prompts.txt"), "rb") as f:
        prompts = [l.rstrip(b"\n") for l in f.read().split(b"\n") if l]
    batch3 = ["你好世界", "こんにちは、世界！", "hello world"]   # test_batch_encode.cpp:39-43
    with open(os.path.join(REF, "examples", "sample_client_texts.txt"), "rb") as f:
        sample = [l.rstrip(b"\n") for l in f.read().split(b"\n") if l][:120]
    texts = prompts + [s.encode() for s in batch3] + sample + edge_texts()
    cases = []
    for n_max in (512, 16):
        ids = reftok_ids(vocab, texts, n_max)
        for s, t in zip(texts, ids):
            cases.append({"text_hex": s.hex(), "n_max_tokens": n_max, "ids": t})
    return {"vocab": vocab, "cases": cases,
            "source": "reference bert.cpp:195-417 compiled by oracle/build_ref.sh"}


def write_vocab_file(path, vocab):
    with open(path, "w", encoding="utf-8") as f:
        for w in vocab:
            f.write(w + "\n")


def make_tiny_model(dirname, vocab, hidden, heads, inter, layers, max_pos, seed):
    import torch
    from transformers import BertConfig, BertModel, BertTokenizerFast
    os.makedirs(dirname, exist_ok=True)
    write_vocab_file(os.path.join(dirname, "vocab.txt"), vocab)
    tok = BertTokenizerFast(vocab_file=os.path.join(dirname, "vocab.txt"))
    tok.save_pretrained(dirname)
    cfg = BertConfig(vocab_size=len(vocab), hidden_size=hidden, num_attention_heads=heads,
                     intermediate_size=inter, num_hidden_layers=layers, max_position_embeddings=max_pos,
                     hidden_act="gelu_pytorch_tanh", layer_norm_eps=1e-5, initializer_range=0.08)
    torch.manual_seed(seed)
    model = BertModel(cfg)
    with torch.no_grad():   # non-trivial LN affine parameters
        for n, p in model.named_parameters():
            if "LayerNorm.weight" in n:
                p.copy_(1.0 + 0.1 * torch.randn_like(p))
            elif n.endswith("bias"):
                p.copy_(0.05 * torch.randn_like(p))
    model.save_pretrained(dirname)
    return model


def torch_embed(model, ids_list):
    """Independent float oracle: HF BertModel + masked mean pool + L2 norm."""
    import torch
    L = max(len(x) for x in ids_list)
    ids = torch.full((len(ids_list), L), 101, dtype=torch.long)
    mask = torch.zeros((len(ids_list), L), dtype=torch.long)
    for i, x in enumerate(ids_list):
        ids[i, : len(x)] = torch.tensor(x)
        mask[i, : len(x)] = 1
    model.eval()
    with torch.no_grad():
        h = model(input_ids=ids, attention_mask=mask, token_type_ids=torch.zeros_like(ids)).last_hidden_state
        m = mask.unsqueeze(-1).float()
        e = (h * m).sum(1) / m.sum(1)
        e = e / e.norm(dim=-1, keepdim=True)
    return e.numpy().astype(np.float32)


def main():
    subprocess.check_call([os.path.join(ROOT, "oracle", "build_ref.sh")])
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    vocab = build_vocab()
    tg = make_tokenizer_golden(vocab)
    with open(os.path.join(HERE, "tokenizer_cases.json"), "w") as f:
        json.dump(tg, f, ensure_ascii=False, indent=0)
    print("tokenizer cases:", len(tg["cases"]), "vocab:", len(vocab))

    env = dict(os.environ, HF_HUB_OFFLINE="1", TRANSFORMERS_OFFLINE="1")
    rng = np.random.default_rng(5)
    specs = {"tiny32": dict(hidden=64, heads=2, inter=128, layers=2, max_pos=128, seed=1),
             "tiny64": dict(hidden=64, heads=1, inter=128, layers=2, max_pos=512, seed=2)}
    for name, sp in specs.items():
        tmp = tempfile.mkdtemp(prefix="hf_" + name + "_")
        model = make_tiny_model(tmp, vocab, **sp)
        for ft in ("0", "1"):    # the reference converter, run on a LOCAL directory only
            subprocess.check_call([sys.executable, os.path.join(REF, "models", "convert-to-ggml.py"), tmp, ft],
                                  env=env, stdout=subprocess.DEVNULL)
        dst = os.path.join(HERE, name)
        os.makedirs(dst, exist_ok=True)
        for fn in ("ggml-model-f32.bin", "ggml-model-f16.bin"):
            shutil.copy(os.path.join(tmp, fn), os.path.join(dst, fn))
        # forward goldens: reference-tokenized texts + random id lists of ragged length
        texts = [bytes.fromhex(c["text_hex"]) for c in tg["cases"] if c["n_max_tokens"] == 512][:12]
        ids = reftok_ids(vocab, texts, sp["max_pos"])
        ids = [x for x in ids if len(x) <= sp["max_pos"]]
        for L in (3, 17, 64, sp["max_pos"]):
            ids.append([101] + [int(v) for v in rng.integers(104, len(vocab), L - 2)] + [102])
        emb_t = torch_embed(model, ids)
        orc = oracle_lib.Oracle(os.path.join(dst, "ggml-model-f32.bin"))
        emb_o = orc.forward_batch(ids, n_threads=8)
        cos = (emb_t * emb_o).sum(-1)
        print(name, "oracle vs torch cosine min", cos.min())
        flat = np.concatenate([np.asarray(x, np.int32) for x in ids])
        lens = np.asarray([len(x) for x in ids], np.int32)
        np.savez_compressed(os.path.join(dst, "forward_f32.npz"), ids=flat, lens=lens,
                            torch_emb=emb_t, oracle_emb=emb_o)
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main()

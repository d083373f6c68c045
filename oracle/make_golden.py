#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE's own code.

CONTAINER-ONLY test infrastructure.  Needs /root/reference (read-only), the `regex` and
`tokenizers` modules and the built libraries (shredword_amd/libshredword_hip.so for the
deterministic synthetic corpora, oracle/_ref/libtrainer.so for the reference trainer).
Only the OUTPUT (data: merge tables, inputs, expected ids) is committed; no reference source.

Expected values come from the reference's primitives, imported by file path from
/root/reference/shredword/base.py (importing the package would dlopen its trainer library,
shredword/__init__.py:1):
  apply_regex  base.py:38-58   get_stats base.py:10-20   merge base.py:22-36
  build_vocab  base.py:60-79   BaseTokenizer.save/load base.py:111-149
composed into the only encode loop they support:
  for chunk in apply_regex(text): ids = list(chunk.encode()); while len(ids) >= 2:
      pair = min(get_stats(ids), key=lambda p: merges.get(p, inf)); stop if pair not in merges;
      ids = merge(ids, pair, merges[pair])

Merge tables:
  toy500.model  500 merges, trained by the reference C++ trainer (shredword/csrc/bpe/bpe.cpp,
                built from its sources by `make -C oracle ref`) on the seeded 10 MB ASCII corpus;
                BPETrainer(target_vocab_size=756, unk_id=0, character_coverage=0.9999,
                min_pair_freq=2) as in SURVEY.md §8c.  toy500.bin is its raw binary output.
  bl32k.model / bl50k.model  32 000 / 50 000 byte-level merges trained with HF `tokenizers`
                (BpeTrainer + ByteLevel, GPT-2 regex) on separate seeded MIXED samples,
                converted to shredword ids (byte b -> id b, merge k -> id 256 + k).
"""
import ctypes
import importlib.util
import json
import os
import random
import subprocess
import sys
import tempfile

import numpy as np
import regex

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
REF_BASE = "/root/reference/shredword/base.py"
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True

from shredword_amd import corpus  # noqa: E402  (synthetic inputs only)

GPT2_DOC_PATTERN = r"""'(?:[sdmt]|ll|ve|re)| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"""  # base.py:46


def load_ref():
    spec = importlib.util.spec_from_file_location("shredword_ref_base", REF_BASE)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


REF = load_ref()


# ------------------------------------------------------------------------------------------
# the reference encode loop, composed from the reference primitives only
# ------------------------------------------------------------------------------------------
def ref_encode_chunk(ids, merges):
    while len(ids) >= 2:
        stats = REF.get_stats(ids)
        pair = min(stats, key=lambda p: merges.get(p, float("inf")))
        if pair not in merges:
            break
        ids = REF.merge(ids, pair, merges[pair])
    return ids


def ref_chunks(text, pattern):
    if pattern == "cl100k":
        return REF.apply_regex(text)
    if pattern == "gpt2":
        return regex.findall(GPT2_DOC_PATTERN, text)
    return [text] if text else []


def ref_encode(text, merges, pattern):
    out = []
    for ch in ref_chunks(text, pattern):
        out.extend(ref_encode_chunk(list(ch.encode("utf-8")), merges))
    return out


# ------------------------------------------------------------------------------------------
# merge tables
# ------------------------------------------------------------------------------------------
def write_v1(path, pairs, pattern=""):
    with open(path, "w") as f:
        f.write("shredword v1\n%s\n0\n" % pattern)
        for a, b in pairs:
            f.write("%d %d\n" % (a, b))


def train_toy500():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"])
    lib = os.path.join(ROOT, "oracle", "_ref", "libtrainer.so")
    buf, off = corpus.synth(1001, corpus.ASCII, 10000, 1000)
    with tempfile.TemporaryDirectory() as td:
        cpath = os.path.join(td, "corpus.txt")
        with open(cpath, "wb") as f:
            f.write(bytes(buf))
        mpath, vpath = os.path.join(td, "toy.model"), os.path.join(td, "toy.vocab")
        # run in a child so the trainer's printf chatter stays out of our output
        code = f"""
import ctypes
L = ctypes.CDLL({lib!r})
class Cfg(ctypes.Structure):
    _fields_ = [("target_vocab_size", ctypes.c_size_t), ("unk_id", ctypes.c_int32),
                ("character_coverage", ctypes.c_float), ("min_pair_freq", ctypes.c_uint64)]
L.create_trainer.restype = ctypes.c_void_p
L.create_trainer.argtypes = [ctypes.POINTER(Cfg)]
L.bpe_load_corpus.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
L.bpe_train.argtypes = [ctypes.c_void_p]
L.bpe_save.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]
c = Cfg(756, 0, 0.9999, 2)
t = L.create_trainer(ctypes.byref(c))
assert L.bpe_load_corpus(t, {cpath!r}.encode()) == 0
assert L.bpe_train(t) > 0
L.bpe_save(t, {mpath!r}.encode(), {vpath!r}.encode())
"""
        subprocess.check_call([sys.executable, "-c", code], stdout=subprocess.DEVNULL)
        raw = open(mpath, "rb").read()
    with open(os.path.join(GOLD, "toy500.bin"), "wb") as f:
        f.write(raw)
    rows = np.frombuffer(raw, dtype="<i4").reshape(-1, 3)
    assert (rows[:, 2] == 256 + np.arange(len(rows))).all()
    write_v1(os.path.join(GOLD, "toy500.model"), [(int(a), int(b)) for a, b, _ in rows])
    return len(rows)


def bytes_to_unicode():
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {chr(c): b for b, c in zip(bs, cs)}


def train_byte_level(n_merges, seed, n_strings, name):
    from tokenizers import Tokenizer, models, pre_tokenizers, trainers
    buf, off = corpus.synth(seed, corpus.MIXED, n_strings, 1074)
    data = bytes(buf)
    texts = (data[off[i]:off[i + 1]].decode("utf-8") for i in range(n_strings))
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    tr = trainers.BpeTrainer(vocab_size=256 + n_merges, min_frequency=2, show_progress=False,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet(), special_tokens=[])
    tok.train_from_iterator(texts, tr)
    raw = json.loads(tok.to_str())["model"]["merges"]
    u2b = bytes_to_unicode()
    ids = {bytes([b]): b for b in range(256)}
    pairs = []
    for k, m in enumerate(raw):
        a, b = m if isinstance(m, list) else m.split(" ")
        ab, bb = bytes(u2b[c] for c in a), bytes(u2b[c] for c in b)
        pairs.append((ids[ab], ids[bb]))
        ids[ab + bb] = 256 + k
    assert len(pairs) == n_merges, (name, len(pairs))
    # well-formed: every pair's members precede its own id
    assert all(a < 256 + k and b < 256 + k for k, (a, b) in enumerate(pairs))
    write_v1(os.path.join(GOLD, name + ".model"), pairs)
    return len(pairs)


def load_merges(name):
    t = REF.BaseTokenizer()
    t.load(os.path.join(GOLD, name + ".model"))
    return t.merges


# ------------------------------------------------------------------------------------------
# fixtures
# ------------------------------------------------------------------------------------------
EDGE = [
    "", " ", "  ", "\n", "\n\n\n", "\r\n", " \r\n ", "a", "aa", "aaa", "aaaa", "aaaaa", "aaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaa",
    "Hello world's 12345 \n\n  x", "I'LL WE'VE THEY'RE it'S don't ſ'ſ 'S", "$$$ hello!!!\n\n", "1234567 89 0.5",
    "a b c　d", "中文字符 測試 漢字", "😀😀 👨‍👩‍👧 x", "é ñ", "ᲉꟋ\U00010ec2 new letters",
    "tab\tsep\tvalues\n", "   leading and trailing   ", "(quoted) \"text\" -- dash...", "mixed 中 and 😀 in 1 line\r\n",
    "\x00\x01\x1c\x1f control", "x" * 40 + " " + "y" * 17, " " * 40, "!" * 30 + "\n",
]


def random_unicode(rng, n):
    pool = [chr(c) for c in list(range(0x20, 0x7F)) + [9, 10, 13, 11, 12, 0x1C, 0x85, 0xA0, 0x17F, 0x1680, 0x2000,
                                                      0x2028, 0x3000, 0x4E00, 0x4E8C, 0x1F600, 0xE9, 0x301, 0x660,
                                                      0x1C89, 0xA7CB, 0x10EC2, 0x2160, 0xFF21]]
    return "".join(rng.choice(pool) for _ in range(n))


def save_encode_fixture(name, texts, merges, pattern, model):
    datas = [t.encode("utf-8") for t in texts]
    off = np.zeros(len(datas) + 1, dtype=np.int64)
    np.cumsum([len(d) for d in datas], out=off[1:])
    ids, ids_off = [], [0]
    for t in texts:
        r = ref_encode(t, merges, pattern)
        ids.extend(r)
        ids_off.append(len(ids))
    np.savez_compressed(os.path.join(GOLD, "enc_%s.npz" % name),
                        bytes=np.frombuffer(b"".join(datas), dtype=np.uint8), off=off,
                        ids=np.array(ids, dtype=np.int32), ids_off=np.array(ids_off, dtype=np.int64))
    return {"file": "enc_%s.npz" % name, "model": model, "pattern": pattern, "n_strings": len(texts),
            "n_bytes": int(off[-1]), "n_tokens": len(ids)}


def corpus_texts(seed, kind, n, mean, max_bytes):
    buf, off = corpus.synth(seed, kind, n, mean)
    data = bytes(buf)
    out, tot = [], 0
    for i in range(n):
        s = data[off[i]:off[i + 1]].decode("utf-8")
        if tot + len(s) > max_bytes:
            break
        out.append(s)
        tot += len(s)
    return out


def primitives_fixture():
    rng = random.Random(7)
    kat = {
        "get_stats": [], "merge": [], "apply_regex_cl100k": [], "apply_regex_gpt2": [], "build_vocab": None,
        "render_token": [],
    }
    for ids in ([1, 2, 3, 1, 2], [], [5], [7, 7, 7, 7], [1, 2, 1, 2, 1], [3, 1, 2, 3, 1, 2, 2]):
        kat["get_stats"].append({"ids": ids, "stats": [[a, b, c] for (a, b), c in REF.get_stats(ids).items()]})
    for ids, pair, idx in (([1, 2, 3, 1, 2], (1, 2), 4), ([97] * 3, (97, 97), 256), ([97] * 4, (97, 97), 256),
                           ([97] * 5, (97, 97), 256), ([1, 1, 2, 1, 1, 1], (1, 1), 9), ([], (1, 2), 3),
                           ([1], (1, 2), 3), ([1, 2], (2, 1), 3)):
        kat["merge"].append({"ids": ids, "pair": list(pair), "idx": idx, "out": REF.merge(ids, pair, idx)})
    texts = EDGE + [random_unicode(rng, rng.randint(0, 48)) for _ in range(400)]
    for t in texts:
        kat["apply_regex_cl100k"].append({"text": t, "chunks": REF.apply_regex(t)})
        kat["apply_regex_gpt2"].append({"text": t, "chunks": regex.findall(GPT2_DOC_PATTERN, t)})
    m = {(104, 101): 256, (256, 108): 257, (257, 108): 258, (258, 111): 259}
    sp = {"<|endoftext|>": 300, "<pad>": 301}
    v = REF.build_vocab(m, sp)
    kat["build_vocab"] = {"merges": [[a, b, i] for (a, b), i in m.items()], "special": [[k, i] for k, i in sp.items()],
                          "vocab": [[i, list(b)] for i, b in v.items()]}
    for t in (b"hello", b"\n\t", b"\xff\xfe", "é中".encode(), b"a\x00b"):
        kat["render_token"].append({"bytes": list(t), "out": REF.render_token(t)})
    # save/load round trip through the reference BaseTokenizer
    with tempfile.TemporaryDirectory() as td:
        model = os.path.join(td, "t.model")
        with open(model, "w", encoding="utf-8") as f:
            f.write("shredword v1\n  some pattern  \n2\n<|endoftext|> 900\n<pad> 901\n"
                    "104 101\n256 108\n32 104\n257 111\n32 104\n")
        t = REF.BaseTokenizer()
        t.load(model)
        kat["load"] = {"text": open(model, encoding="utf-8").read(), "pattern": t.pattern,
                       "merges": [[a, b, i] for (a, b), i in t.merges.items()],
                       "special": [[k, i] for k, i in t.special_tokens.items()],
                       "vocab": [[i, list(b)] for i, b in t.vocab.items()]}
        t.save(os.path.join(td, "out"))
        # a duplicated pair whose first id is referenced later: build_vocab raises KeyError
        with open(model, "w", encoding="utf-8") as f:
            f.write("shredword v1\n\n0\n104 101\n256 108\n104 101\n")
        try:
            REF.BaseTokenizer().load(model)
            kat["load_error"] = {"text": open(model).read(), "error": None}
        except Exception as e:  # noqa: BLE001
            kat["load_error"] = {"text": open(model).read(), "error": type(e).__name__}
        kat["save"] = {"model": open(os.path.join(td, "out.model"), encoding="utf-8").read(),
                       "vocab": open(os.path.join(td, "out.vocab"), encoding="utf-8").read()}
    with open(os.path.join(GOLD, "primitives.json"), "w", encoding="utf-8") as f:
        json.dump(kat, f, ensure_ascii=True, indent=0)


def main():
    os.makedirs(GOLD, exist_ok=True)
    info = {"regex": regex.__version__, "reference": REF_BASE, "fixtures": []}
    import tokenizers
    info["tokenizers"] = tokenizers.__version__
    info["toy500_merges"] = train_toy500()
    info["bl32k_merges"] = train_byte_level(32000, 2002, 30000, "bl32k")
    info["bl50k_merges"] = train_byte_level(50000, 2003, 60000, "bl50k")
    primitives_fixture()
    rng = random.Random(11)
    m500, m32, m50 = load_merges("toy500"), load_merges("bl32k"), load_merges("bl50k")
    fx = info["fixtures"]
    fx.append(save_encode_fixture("toy500_ascii", EDGE + corpus_texts(3001, corpus.ASCII, 400, 1000, 200_000),
                                  m500, "cl100k", "toy500.model"))
    fx.append(save_encode_fixture("bl32k_mixed", EDGE + corpus_texts(3002, corpus.MIXED, 400, 1074, 250_000)
                                  + [random_unicode(rng, rng.randint(0, 200)) for _ in range(200)],
                                  m32, "cl100k", "bl32k.model"))
    fx.append(save_encode_fixture("bl32k_gpt2", EDGE + corpus_texts(3004, corpus.MIXED, 100, 1074, 60_000),
                                  m32, "gpt2", "bl32k.model"))
    fx.append(save_encode_fixture("bl32k_none", EDGE + corpus_texts(3005, corpus.MIXED, 40, 60, 2_000),
                                  m32, "none", "bl32k.model"))
    stress = corpus_texts(3003, corpus.STRESS, 600, 600, 200_000)
    longs = [s for s in stress if len(s) == 4096][:2]
    stress = [s for s in stress if len(s) != 4096] + longs
    fx.append(save_encode_fixture("bl50k_stress", EDGE + stress, m50, "cl100k", "bl50k.model"))
    # an ill-formed user table: random pairs, duplicate values, ids referencing later ids
    r = random.Random(5)
    alpha = b"abcde "
    bad = {}
    for _ in range(400):
        bad[(r.choice(list(alpha) + list(range(256, 300))), r.choice(list(alpha) + list(range(256, 300))))] = r.randint(256, 299)
    with open(os.path.join(GOLD, "illformed.json"), "w") as f:
        json.dump([[a, b, v] for (a, b), v in bad.items()], f)
    texts = ["".join(r.choice("abcde ") for _ in range(r.randint(0, 60))) for _ in range(300)]
    fx.append(save_encode_fixture("illformed", texts, bad, "none", "illformed.json"))
    with open(os.path.join(GOLD, "index.json"), "w") as f:
        json.dump(info, f, indent=1)
    print(json.dumps(info, indent=1))


if __name__ == "__main__":
    main()

"""CPU-side checks of the boundary and the host logic (no GPU needed).

* libgpubpe.so loads and exports every symbol include/gpubpe.h declares;
* the host-side Vocab / trie compiler of the product match the reference's
  own vocab.js / trie.js outputs (tests/golden/ref_modules.json);
* without a HIP device the API fails loudly (no CPU fallback).
"""
import ctypes as C
import json
import os
import re

import pytest

import sys

from conftest import GOLDEN, ROOT

HEADER = os.path.join(ROOT, "include", "gpubpe.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(gbpe_[a-z0-9_]+)\s*\(", src)
    return sorted(set(n for n in names if not n.endswith("_cb")))


@pytest.fixture(scope="module")
def lib():
    from gpubpe import _lib
    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return _lib.load()


def test_header_declares_the_boundary():
    names = _declared_functions()
    for must in ("gbpe_ctx_create", "gbpe_train", "gbpe_trainer_step", "gbpe_trie_upload", "gbpe_encode",
                 "gbpe_last_error", "gbpe_word_boundary"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in _declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    from gpubpe import _lib
    assert set(_declared_functions()) <= set(_lib.EXPORTED)


def test_kernel_inventory(lib):
    n = lib.gbpe_kernel_count()
    names = [lib.gbpe_kernel_name(i).decode() for i in range(n)]
    assert "k_delta" in names and "k_trie_walk" in names and len(names) == len(set(names))
    assert lib.gbpe_version().startswith(b"gpubpe")


def test_abi_version_and_stats_layout(lib):
    """The header's ABI version is the library's, and the ctypes mirror of
    gbpe_trainer_stats has the C struct's size (a stale caller struct would be
    overrun by gbpe_trainer_stats_get)."""
    from gpubpe import _lib
    src = open(HEADER).read()
    want = int(re.search(r"#define GBPE_ABI_VERSION (\d+)", src).group(1))
    assert lib.gbpe_abi_version() == want
    assert f"abi {want}".encode() in lib.gbpe_version()
    assert lib.gbpe_trainer_stats_size() == C.sizeof(_lib.TrainerStats)


def test_no_device_fails_loudly(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    from gpubpe import BPEEngine, _lib
    with pytest.raises(_lib.GpuBpeError):
        BPEEngine().init()


def test_product_vocab_matches_reference_vocab_js():
    from gpubpe import Vocab
    ref = json.load(open(os.path.join(GOLDEN, "ref_modules.json")))
    for inp, out in zip(ref["inputs"]["vocab_cases"], ref["outputs"]["vocab_cases"]):
        v = Vocab()
        ids = [v.add_merge(a, b) for a, b in inp["merges"]]
        assert ids == out["ids"]
        assert v.entries == out["entries"] and v.strings == out["strings"]
        assert v.export() == out["export"]


def test_product_trie_matches_reference_trie_js():
    from gpubpe import compile_vocab_to_trie, parse_header, parse_trie_buffers
    ref = json.load(open(os.path.join(GOLDEN, "ref_modules.json")))
    for inp, out in zip(ref["inputs"]["trie_cases"], ref["outputs"]["trie_cases"]):
        blob = compile_vocab_to_trie(inp["vocab"])
        assert blob.hex() == out["trie_hex"], inp["name"]
        h = parse_header(blob)
        assert h == out["header"]
        nodes, edges = parse_trie_buffers(blob, h)
        assert nodes.tolist() == out["nodes"] and edges.tolist() == out["edges"]


def test_trie_parse_errors():
    from gpubpe import parse_header
    with pytest.raises(ValueError, match="magic"):
        parse_header(b"\0" * 28)
    import struct
    with pytest.raises(ValueError, match="version"):
        parse_header(struct.pack("<7I", 0x54524945, 9, 0, 0, 0, 0, 0))


def test_dxft_pack_matches_oracle():
    """gbpe_dxft_pack (native .bin writer) == the oracle's restatement of export-controller.js:221-248."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bpe_oracle as O
    from gpubpe.export import dxft_bin
    vocab_export = {"version": 1, "vocabSize": 259, "vocab": [[i] for i in range(256)] + [[116, 104], [104], []],
                    "merges": [[116, 104, 256]]}
    for toks in ([], [1, 2, 3, 256, 65535], list(range(1000))):
        assert dxft_bin(toks, 259, vocab_export) == O.dxft_bin(toks, 259, vocab_export)
    assert dxft_bin([5], 256, None) == O.dxft_bin([5], 256, None)


def test_model_json_round_trip():
    from gpubpe.export import load_model_json, model_json
    model = {"vocabSize": 258, "vocab": [[i] for i in range(256)] + [[104, 105], [0xE2, 0x82]],
             "merges": [[104, 105, 256, 7], [0xE2, 0x82, 257, 3]]}
    s = model_json(model)
    assert s.startswith('{"version":1,"vocabSize":258,"vocab":[[0],[1],')     # JSON.stringify layout
    m = load_model_json(s)
    assert m["vocabSize"] == 258 and m["merges"] == [[104, 105, 256], [0xE2, 0x82, 257]]
    assert m["vocabStrings"][256] == "hi" and m["vocabStrings"][257] == "�"   # non-fatal UTF-8 decode
    with pytest.raises(ValueError, match="missing vocab or merges"):
        load_model_json({"vocab": [[1]]})

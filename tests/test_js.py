"""Node.js host (N-API addon + JS modules keeping the reference API).

CPU: the JS Vocab / trie modules reproduce the reference vocab.js / trie.js
goldens.  GPU: BPETrainer / TrieTokenizer through the addon equal the oracle.
"""
import base64
import json
import os
import shutil
import subprocess

import pytest

import bpe_oracle as O
from conftest import ROOT

NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def _run(script, *args):
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", script), *args], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_js_host_modules_match_reference_goldens():
    assert _run("test_host.mjs").startswith("ok")


@pytest.mark.gpu
def test_js_addon_train_and_encode(tmp_path):
    addon = os.path.join(ROOT, "gpu-bpe_amd", "js", "gpubpe.node")
    assert os.path.exists(addon), "build the addon: make -C gpu-bpe_amd addon"
    from gpubpe import synth
    cases = []
    for name, data, target, text, cs in (
            ("english", synth.english(40000, seed=41), 600, synth.english(30000, seed=42), None),
            ("multilingual", synth.multilingual(40000, seed=43), 500, synth.multilingual(30000, seed=44), 64)):
        ref = O.train(data, target)
        merges = [m[:3] for m in ref["merges"]]
        voc = O.vocab_from_merges(merges)
        blob = O.compile_vocab_to_trie(voc.entries)
        hdr = O.parse_header(blob)
        nodes, edges = O.parse_trie_buffers(blob, hdr)
        chunk = cs or O.adaptive_chunk_size(hdr["maxTokenLen"])
        toks = O.encode_chunked(text, nodes, edges, chunk).tolist()
        cases.append({"name": name, "b64": base64.b64encode(data).decode(), "target": target, "merges": merges,
                      "export": voc.export(), "text_b64": base64.b64encode(text).decode(), "chunkSize": cs,
                      "tokens": toks})
    code = synth.code(30000, seed=45)
    ws = O.gpt4_word_starts(code)
    pre = {"b64": base64.b64encode(code).decode(), "word_starts": ws.tolist(), "target": 500,
           "merges": [m[:3] for m in O.train(code, 500, word_starts=ws)["merges"]]}
    me_text = synth.english(8000, seed=46)
    me_merges = cases[0]["merges"]
    me = {"merges": me_merges, "text": me_text.decode("utf-8", "replace"),
          "tokens": O.encode_merge_order(me_text.decode("utf-8", "replace").encode(), me_merges)}
    p = tmp_path / "cases.json"
    p.write_text(json.dumps({"train": cases, "pretok": pre, "merge_encode": me}))
    assert _run("test_gpu.mjs", str(p)).strip().splitlines()[-1].startswith("ok")

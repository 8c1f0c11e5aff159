"""gpubpe — MI355X-native BPE training merge loop + chunked trie encode.

Python host binding over the C-ABI library ``lib/libgpubpe.so`` (HIP,
gfx950).  Mirrors the reference toprakdeviren/gpu-bpe JavaScript API:
BPEEngine (engine.js), BPETrainer (trainer.js), TrieTokenizer
(tokenizer/tokenizer.js), Vocab (vocab.js), trie compile/parse (trie.js).
"""
from .engine import BPEEngine, INVALID_TOKEN, MAX_WG_DIM, TABLE_SIZE, WORKGROUP_SIZE  # noqa: F401
from .pretokenizer import GpuPreTokenizer  # noqa: F401
from .merge_encoder import MergeEncoder  # noqa: F401
from .tokenizer import TrieTokenizer  # noqa: F401
from .trainer import BATCH_SIZE, BPETrainer  # noqa: F401
from .trie import compile_vocab_to_trie, parse_header, parse_trie_buffers  # noqa: F401
from .vocab import Vocab  # noqa: F401

export { BPEEngine, WORKGROUP_SIZE, TABLE_SIZE, INVALID_TOKEN, MAX_WG_DIM, GPU_LIMITS, dispatch2D } from './engine.js';
export { BPETrainer, BATCH_SIZE } from './trainer.js';
export { TrieTokenizer } from './tokenizer.js';
export { Vocab, displayString } from './vocab.js';
export { compileVocabToTrie, parseHeader, parseTrieBuffers } from './trie.js';
export { GpuPreTokenizer } from './pretokenizer.js';
export { modelToJSON, loadModelJSON, dxftBin, exportDXFT } from './export.js';
export { MergeEncoder } from './merge-encoder.js';

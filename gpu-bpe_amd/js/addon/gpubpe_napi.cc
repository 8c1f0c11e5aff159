// Node.js N-API addon over the gpubpe C-ABI (include/gpubpe.h).
//
// This is the native half of the drop-in for the reference's device layer
// (src/bpe/engine.js + WGSL).  The JS modules beside it (engine.js,
// trainer.js, tokenizer.js) keep the reference's API.  Long-running calls
// (trainer steps, encode) run as napi_async_work off the JS thread and
// resolve Promises, so the event loop never blocks — the role the Web
// Worker + yieldToEventLoop play in the reference (bpe-worker.js,
// trainer.js:39-41, 317).
//
// Exports:
//   createContext(device) -> ctx                 limits(ctx) -> {maxBufferSize}
//   kernelNames() -> string[]                    destroyContext(ctx)
//   trainerCreate(ctx, bytes, wordStarts|null, {targetVocabSize, vocabSize, nextTokenId, batchSize, exact}) -> trainer
//   trainerStep(trainer, maxMerges) -> Promise<{merges: Uint32Array [a,b,id,count]*, earlyStop, symbolCount}>
//   trainerDestroy(trainer)
//   trieUpload(ctx, nodes: Uint32Array, edges: Uint32Array) -> trie      trieFree(trie)
//   encode(ctx, trie, bytes, chunkSize) -> Promise<Uint32Array>
//   wordBoundary(ctx, bytes) -> Uint8Array
//
// Concurrency and lifetimes.  Every call that touches a context's device state
// (its stream, pooled encode buffers, error string) holds that context's mutex,
// so overlapping Promises (Promise.all over encode / trainerStep) run one after
// the other on the device instead of racing (the reference serialises them on
// one WebGPU queue).  Contexts are reference-counted by their trainers, tries,
// BPE tables and in-flight work: destroyContext() closes a context for new
// calls, and the device context is freed when the last of those is gone.
// trainerDestroy() / trieFree() during a step / encode defer the free to its
// completion.
#include <node_api.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "gpubpe.h"

#define NAPI_CALL(env, call)                                                       \
    do {                                                                           \
        if ((call) != napi_ok) {                                                   \
            napi_throw_error((env), nullptr, "gpubpe addon: N-API call failed");   \
            return nullptr;                                                        \
        }                                                                          \
    } while (0)

namespace {

// All reference counts below change on the JS thread only (calls, finalizers,
// async-work completions); worker threads only take `mu`.
struct Ctx {
    gbpe_ctx* ctx = nullptr;
    std::mutex mu;          // serialises device work on this context
    int refs = 1;           // the JS external + children + in-flight work
    bool closed = false;    // destroyContext() was called
    bool js_ref = true;     // the JS external's reference is still held
};
void ctx_release(Ctx* c) {
    if (c && --c->refs == 0) {
        if (c->ctx) gbpe_ctx_destroy(c->ctx);
        delete c;
    }
}
bool ctx_usable(const Ctx* c) { return c && c->ctx && !c->closed; }

struct Trainer {
    gbpe_trainer* t = nullptr;
    Ctx* owner = nullptr;
    uint32_t batch = 128;
    int inflight = 0;              // queued / running trainerStep works
    bool destroy_pending = false;  // trainerDestroy() while a step ran
};
void trainer_free(Trainer* t) {   // the device trainer and its context reference
    if (t->t) {
        std::lock_guard<std::mutex> g(t->owner->mu);
        gbpe_trainer_destroy(t->t);
        t->t = nullptr;
    }
    if (t->owner) {
        ctx_release(t->owner);
        t->owner = nullptr;
    }
}
struct Trie {
    gbpe_trie* trie = nullptr;
    Ctx* owner = nullptr;
    int inflight = 0;
    bool destroy_pending = false;
};
void trie_free(Trie* t) {
    if (t->trie) {
        std::lock_guard<std::mutex> g(t->owner->mu);
        gbpe_trie_free(t->trie);
        t->trie = nullptr;
    }
    if (t->owner) {
        ctx_release(t->owner);
        t->owner = nullptr;
    }
}

std::string last_error(gbpe_ctx* c, const char* what, int rc) {
    std::string m = what;
    m += ": ";
    const char* e = c ? gbpe_last_error(c) : nullptr;
    m += (e && *e) ? e : "gpubpe error";
    m += " (status " + std::to_string(rc) + ")";
    return m;
}

napi_value throw_status(napi_env env, gbpe_ctx* c, const char* what, int rc) {
    napi_throw_error(env, nullptr, last_error(c, what, rc).c_str());
    return nullptr;
}

template <typename T>
T* unwrap_external(napi_env env, napi_value v) {
    void* p = nullptr;
    if (napi_get_value_external(env, v, &p) != napi_ok) return nullptr;
    return static_cast<T*>(p);
}

bool get_bytes(napi_env env, napi_value v, const uint8_t** data, size_t* len) {
    bool is_ta = false;
    napi_is_typedarray(env, v, &is_ta);
    if (!is_ta) return false;
    napi_typedarray_type type;
    size_t length = 0, offset = 0;
    void* raw = nullptr;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &type, &length, &raw, &ab, &offset) != napi_ok) return false;
    if (type != napi_uint8_array) return false;
    *data = static_cast<const uint8_t*>(raw);
    *len = length;
    return true;
}

bool get_u32s(napi_env env, napi_value v, const uint32_t** data, size_t* len) {
    bool is_ta = false;
    napi_is_typedarray(env, v, &is_ta);
    if (!is_ta) return false;
    napi_typedarray_type type;
    size_t length = 0, offset = 0;
    void* raw = nullptr;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &type, &length, &raw, &ab, &offset) != napi_ok) return false;
    if (type != napi_uint32_array) return false;
    *data = static_cast<const uint32_t*>(raw);
    *len = length;
    return true;
}

uint32_t get_u32_prop(napi_env env, napi_value obj, const char* name, uint32_t dflt) {
    bool has = false;
    if (napi_has_named_property(env, obj, name, &has) != napi_ok || !has) return dflt;
    napi_value v;
    napi_get_named_property(env, obj, name, &v);
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t == napi_boolean) {
        bool b = false;
        napi_get_value_bool(env, v, &b);
        return b ? 1u : 0u;
    }
    if (t != napi_number) return dflt;
    uint32_t out = dflt;
    napi_get_value_uint32(env, v, &out);
    return out;
}

napi_value make_u32_array(napi_env env, const uint32_t* src, size_t n) {
    napi_value ab, ta;
    void* dst = nullptr;
    if (napi_create_arraybuffer(env, n * 4, &dst, &ab) != napi_ok) return nullptr;
    if (n) memcpy(dst, src, n * 4);
    if (napi_create_typedarray(env, napi_uint32_array, n, ab, 0, &ta) != napi_ok) return nullptr;
    return ta;
}

// ── context ──────────────────────────────────────────────────────────────

void ctx_finalize(napi_env, void* data, void*) {
    Ctx* c = static_cast<Ctx*>(data);
    if (c->js_ref) {
        c->js_ref = false;
        ctx_release(c);
    }
}

napi_value CreateContext(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    int32_t dev = 0;
    if (argc >= 1) napi_get_value_int32(env, argv[0], &dev);
    auto* c = new Ctx();
    int rc = gbpe_ctx_create(dev, &c->ctx);
    if (rc != GBPE_OK) {
        delete c;
        std::string m = "No usable HIP device " + std::to_string(dev) + " (gbpe_ctx_create status " +
                        std::to_string(rc) + ")";
        napi_throw_error(env, nullptr, m.c_str());
        return nullptr;
    }
    napi_value ext;
    NAPI_CALL(env, napi_create_external(env, c, ctx_finalize, nullptr, &ext));
    return ext;
}

napi_value DestroyContext(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Ctx* c = argc ? unwrap_external<Ctx>(env, argv[0]) : nullptr;
    if (c && !c->closed) {   // freed once its trainers, tries and in-flight work are gone
        c->closed = true;
        if (c->js_ref) {
            c->js_ref = false;
            ctx_release(c);
        }
    }
    return nullptr;
}

napi_value Limits(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Ctx* c = argc ? unwrap_external<Ctx>(env, argv[0]) : nullptr;
    if (!ctx_usable(c)) {
        napi_throw_type_error(env, nullptr, "limits(ctx): invalid context");
        return nullptr;
    }
    uint64_t mb = 0;
    std::unique_lock<std::mutex> g(c->mu);
    int rc = gbpe_ctx_limits(c->ctx, &mb);
    g.unlock();
    if (rc != GBPE_OK) return throw_status(env, c->ctx, "limits", rc);
    napi_value obj, v;
    NAPI_CALL(env, napi_create_object(env, &obj));
    NAPI_CALL(env, napi_create_double(env, (double)mb, &v));
    NAPI_CALL(env, napi_set_named_property(env, obj, "maxBufferSize", v));
    return obj;
}

napi_value KernelNames(napi_env env, napi_callback_info) {
    napi_value arr;
    const int n = gbpe_kernel_count();
    NAPI_CALL(env, napi_create_array_with_length(env, n, &arr));
    for (int i = 0; i < n; ++i) {
        napi_value s;
        NAPI_CALL(env, napi_create_string_utf8(env, gbpe_kernel_name(i), NAPI_AUTO_LENGTH, &s));
        NAPI_CALL(env, napi_set_element(env, arr, i, s));
    }
    return arr;
}

napi_value WordBoundary(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Ctx* c = argc >= 1 ? unwrap_external<Ctx>(env, argv[0]) : nullptr;
    const uint8_t* data = nullptr;
    size_t len = 0;
    if (!ctx_usable(c) || argc < 2 || !get_bytes(env, argv[1], &data, &len)) {
        napi_throw_type_error(env, nullptr, "wordBoundary(ctx, Uint8Array)");
        return nullptr;
    }
    napi_value ab, ta;
    void* dst = nullptr;
    NAPI_CALL(env, napi_create_arraybuffer(env, len, &dst, &ab));
    std::unique_lock<std::mutex> g(c->mu);
    int rc = gbpe_word_boundary(c->ctx, data, len, static_cast<uint8_t*>(dst));
    g.unlock();
    if (rc != GBPE_OK) return throw_status(env, c->ctx, "wordBoundary", rc);
    NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, len, ab, 0, &ta));
    return ta;
}

// GPT-4 rule word starts (PreTokenizer.preTokenizeBytes, pre_tokenizer.mjs:459-509)
napi_value PretokenizeGpt4(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Ctx* c = argc >= 1 ? unwrap_external<Ctx>(env, argv[0]) : nullptr;
    const uint8_t* data = nullptr;
    size_t len = 0;
    if (!ctx_usable(c) || argc < 2 || !get_bytes(env, argv[1], &data, &len)) {
        napi_throw_type_error(env, nullptr, "pretokenizeGpt4(ctx, Uint8Array)");
        return nullptr;
    }
    napi_value ab, ta;
    void* dst = nullptr;
    NAPI_CALL(env, napi_create_arraybuffer(env, len, &dst, &ab));
    std::unique_lock<std::mutex> g(c->mu);
    int rc = gbpe_pretokenize_gpt4(c->ctx, data, len, static_cast<uint8_t*>(dst));
    g.unlock();
    if (rc != GBPE_OK) return throw_status(env, c->ctx, "pretokenizeGpt4", rc);
    NAPI_CALL(env, napi_create_typedarray(env, napi_uint8_array, len, ab, 0, &ta));
    return ta;
}

// ── trainer ──────────────────────────────────────────────────────────────

void trainer_finalize(napi_env, void* data, void*) {
    Trainer* t = static_cast<Trainer*>(data);
    trainer_free(t);   // (in-flight steps hold a reference to the external: none runs now)
    delete t;
}

napi_value TrainerCreate(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Ctx* c = argc >= 1 ? unwrap_external<Ctx>(env, argv[0]) : nullptr;
    const uint8_t* data = nullptr;
    size_t len = 0;
    if (!ctx_usable(c) || argc < 4 || !get_bytes(env, argv[1], &data, &len)) {
        napi_throw_type_error(env, nullptr, "trainerCreate(ctx, Uint8Array, wordStarts|null, opts)");
        return nullptr;
    }
    const uint8_t* ws = nullptr;
    size_t wslen = 0;
    napi_valuetype wt;
    napi_typeof(env, argv[2], &wt);
    if (wt != napi_null && wt != napi_undefined) {
        if (!get_bytes(env, argv[2], &ws, &wslen) || wslen != len) {
            napi_throw_type_error(env, nullptr, "wordStarts must be a Uint8Array of the byte length");
            return nullptr;
        }
    }
    gbpe_train_opts o{};
    o.target_vocab_size = get_u32_prop(env, argv[3], "targetVocabSize", 4096);
    o.vocab_size = get_u32_prop(env, argv[3], "vocabSize", 256);
    o.next_token_id = get_u32_prop(env, argv[3], "nextTokenId", 256);
    o.batch_size = get_u32_prop(env, argv[3], "batchSize", GBPE_BATCH_SIZE);
    o.flags = get_u32_prop(env, argv[3], "exact", 0) ? GBPE_TRAIN_EXACT_COMPACTION : 0u;
    auto* t = new Trainer();
    t->batch = o.batch_size ? o.batch_size : GBPE_BATCH_SIZE;
    std::unique_lock<std::mutex> g(c->mu);
    int rc = gbpe_trainer_create(c->ctx, data, len, ws, 0, &o, &t->t);
    g.unlock();
    if (rc == GBPE_OK) {
        t->owner = c;
        ++c->refs;
    } else {
        delete t;
        if (rc == GBPE_E_EMPTY) {
            napi_throw_error(env, nullptr, "No symbols to train on — corpus is empty after pre-processing");
            return nullptr;
        }
        return throw_status(env, c->ctx, "train", rc);
    }
    napi_value ext;
    NAPI_CALL(env, napi_create_external(env, t, trainer_finalize, nullptr, &ext));
    return ext;
}

napi_value TrainerDestroy(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Trainer* t = argc ? unwrap_external<Trainer>(env, argv[0]) : nullptr;
    if (t && t->t) {
        if (t->inflight) t->destroy_pending = true;   // step_complete frees it
        else trainer_free(t);
    }
    return nullptr;
}

struct StepWork {
    napi_async_work work = nullptr;
    napi_deferred deferred = nullptr;
    napi_ref keep = nullptr;   // keeps the trainer external alive while the work runs
    Trainer* tr = nullptr;
    uint32_t max_merges = 0;
    std::vector<uint32_t> merges;
    uint32_t n_done = 0, early = 0;
    uint64_t symbols = 0;
    int rc = GBPE_OK;
    std::string err;
};

void step_execute(napi_env, void* data) {
    auto* w = static_cast<StepWork*>(data);
    w->merges.assign((size_t)w->tr->batch * 4, 0);
    std::lock_guard<std::mutex> g(w->tr->owner->mu);
    w->rc = gbpe_trainer_step(w->tr->t, w->max_merges, w->merges.data(), &w->n_done, &w->early);
    if (w->rc != GBPE_OK) {
        w->err = last_error(w->tr->owner->ctx, "train step", w->rc);
        return;
    }
    gbpe_trainer_stats st;
    if (gbpe_trainer_stats_get(w->tr->t, &st) == GBPE_OK) w->symbols = st.symbol_count;
}

void step_complete(napi_env env, napi_status, void* data) {
    auto* w = static_cast<StepWork*>(data);
    if (w->rc != GBPE_OK) {
        napi_value msg, err;
        napi_create_string_utf8(env, w->err.c_str(), NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, nullptr, msg, &err);
        napi_reject_deferred(env, w->deferred, err);
    } else {
        napi_value obj, v;
        napi_create_object(env, &obj);
        napi_set_named_property(env, obj, "merges", make_u32_array(env, w->merges.data(), (size_t)w->n_done * 4));
        napi_get_boolean(env, w->early != 0, &v);
        napi_set_named_property(env, obj, "earlyStop", v);
        napi_create_double(env, (double)w->symbols, &v);
        napi_set_named_property(env, obj, "symbolCount", v);
        napi_resolve_deferred(env, w->deferred, obj);
    }
    if (--w->tr->inflight == 0 && w->tr->destroy_pending) trainer_free(w->tr);
    napi_delete_reference(env, w->keep);
    napi_delete_async_work(env, w->work);
    delete w;
}

napi_value TrainerStep(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Trainer* t = argc >= 1 ? unwrap_external<Trainer>(env, argv[0]) : nullptr;
    if (!t || !t->t || t->destroy_pending) {
        napi_throw_type_error(env, nullptr, "trainerStep(trainer, maxMerges): invalid trainer");
        return nullptr;
    }
    auto* w = new StepWork();
    w->tr = t;
    ++t->inflight;   // (the trainer holds its context: it outlives the work)
    if (argc >= 2) napi_get_value_uint32(env, argv[1], &w->max_merges);
    napi_value promise, name;
    NAPI_CALL(env, napi_create_promise(env, &w->deferred, &promise));
    NAPI_CALL(env, napi_create_reference(env, argv[0], 1, &w->keep));
    NAPI_CALL(env, napi_create_string_utf8(env, "gpubpe.trainerStep", NAPI_AUTO_LENGTH, &name));
    NAPI_CALL(env, napi_create_async_work(env, nullptr, name, step_execute, step_complete, w, &w->work));
    NAPI_CALL(env, napi_queue_async_work(env, w->work));
    return promise;
}

// ── trie + encode ────────────────────────────────────────────────────────

void trie_finalize(napi_env, void* data, void*) {
    Trie* t = static_cast<Trie*>(data);
    trie_free(t);
    delete t;
}

napi_value TrieUpload(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Ctx* c = argc >= 1 ? unwrap_external<Ctx>(env, argv[0]) : nullptr;
    const uint32_t *nodes = nullptr, *edges = nullptr;
    size_t nn = 0, ne = 0;
    if (!ctx_usable(c) || argc < 3 || !get_u32s(env, argv[1], &nodes, &nn) || !get_u32s(env, argv[2], &edges, &ne)) {
        napi_throw_type_error(env, nullptr, "trieUpload(ctx, nodes: Uint32Array, edges: Uint32Array)");
        return nullptr;
    }
    auto* t = new Trie();
    std::unique_lock<std::mutex> g(c->mu);
    int rc = gbpe_trie_upload(c->ctx, nodes, (uint32_t)(nn / 3), edges, (uint32_t)(ne / 2), &t->trie);
    g.unlock();
    if (rc == GBPE_OK) {
        t->owner = c;
        ++c->refs;
    }
    if (rc != GBPE_OK) {
        delete t;
        return throw_status(env, c->ctx, "trie upload", rc);
    }
    napi_value ext;
    NAPI_CALL(env, napi_create_external(env, t, trie_finalize, nullptr, &ext));
    return ext;
}

napi_value TrieFree(napi_env env, napi_callback_info info) {
    size_t argc = 1;
    napi_value argv[1];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Trie* t = argc ? unwrap_external<Trie>(env, argv[0]) : nullptr;
    if (t && t->trie) {
        if (t->inflight) t->destroy_pending = true;   // encode_complete frees it
        else trie_free(t);
    }
    return nullptr;
}

// ── merge-rank encoder (TokenizerManager.encode, tokenizer-manager.js:13-61) ──

struct Bpe {
    gbpe_bpe* bpe = nullptr;
    Ctx* owner = nullptr;
};

void bpe_finalize(napi_env, void* data, void*) {
    Bpe* b = static_cast<Bpe*>(data);
    if (b->bpe) {
        std::lock_guard<std::mutex> g(b->owner->mu);
        gbpe_bpe_free(b->bpe);
    }
    ctx_release(b->owner);
    delete b;
}

napi_value BpeUpload(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Ctx* c = argc >= 1 ? unwrap_external<Ctx>(env, argv[0]) : nullptr;
    const uint32_t* m = nullptr;
    size_t nm = 0;
    if (!ctx_usable(c) || argc < 2 || !get_u32s(env, argv[1], &m, &nm)) {
        napi_throw_type_error(env, nullptr, "bpeUpload(ctx, merges: Uint32Array [a,b,id]*)");
        return nullptr;
    }
    auto* b = new Bpe();
    std::unique_lock<std::mutex> g(c->mu);
    int rc = gbpe_bpe_upload(c->ctx, m, (uint32_t)(nm / 3), &b->bpe);
    g.unlock();
    if (rc == GBPE_OK) {
        b->owner = c;
        ++c->refs;
    }
    if (rc != GBPE_OK) {
        delete b;
        return throw_status(env, c->ctx, "bpe upload", rc);
    }
    napi_value ext;
    NAPI_CALL(env, napi_create_external(env, b, bpe_finalize, nullptr, &ext));
    return ext;
}

napi_value BpeEncode(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Ctx* c = argc >= 1 ? unwrap_external<Ctx>(env, argv[0]) : nullptr;
    Bpe* b = argc >= 2 ? unwrap_external<Bpe>(env, argv[1]) : nullptr;
    const uint8_t* data = nullptr;
    size_t len = 0;
    if (!ctx_usable(c) || !b || !b->bpe || argc < 3 || !get_bytes(env, argv[2], &data, &len)) {
        napi_throw_type_error(env, nullptr, "bpeEncode(ctx, bpe, Uint8Array)");
        return nullptr;
    }
    std::vector<uint32_t> out(len ? len : 1);
    uint64_t n = 0;
    std::unique_lock<std::mutex> g(c->mu);
    int rc = gbpe_bpe_encode(c->ctx, b->bpe, data, len, out.data(), out.size(), &n);
    g.unlock();
    if (rc != GBPE_OK) return throw_status(env, c->ctx, "bpe encode", rc);
    return make_u32_array(env, out.data(), (size_t)n);
}

struct EncodeWork {
    napi_async_work work = nullptr;
    napi_deferred deferred = nullptr;
    napi_ref keep_in = nullptr, keep_ctx = nullptr, keep_trie = nullptr;
    Ctx* c = nullptr;
    Trie* trie = nullptr;
    const uint8_t* data = nullptr;
    size_t len = 0;
    uint32_t cs = 0;
    std::vector<uint32_t> out;
    uint64_t n_out = 0;
    int rc = GBPE_OK;
    std::string err;
};

void encode_execute(napi_env, void* data) {
    auto* w = static_cast<EncodeWork*>(data);
    w->out.resize(w->len ? w->len : 1);
    std::lock_guard<std::mutex> g(w->c->mu);
    w->rc = gbpe_encode(w->c->ctx, w->trie->trie, w->data, w->len, w->cs, w->out.data(), w->len, &w->n_out);
    if (w->rc != GBPE_OK) w->err = last_error(w->c->ctx, "encode", w->rc);
}

void encode_complete(napi_env env, napi_status, void* data) {
    auto* w = static_cast<EncodeWork*>(data);
    if (w->rc != GBPE_OK) {
        napi_value msg, err;
        napi_create_string_utf8(env, w->err.c_str(), NAPI_AUTO_LENGTH, &msg);
        napi_create_error(env, nullptr, msg, &err);
        napi_reject_deferred(env, w->deferred, err);
    } else {
        napi_resolve_deferred(env, w->deferred, make_u32_array(env, w->out.data(), (size_t)w->n_out));
    }
    if (--w->trie->inflight == 0 && w->trie->destroy_pending) trie_free(w->trie);
    ctx_release(w->c);
    napi_delete_reference(env, w->keep_in);
    napi_delete_reference(env, w->keep_ctx);
    napi_delete_reference(env, w->keep_trie);
    napi_delete_async_work(env, w->work);
    delete w;
}

napi_value Encode(napi_env env, napi_callback_info info) {
    size_t argc = 4;
    napi_value argv[4];
    NAPI_CALL(env, napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    Ctx* c = argc >= 1 ? unwrap_external<Ctx>(env, argv[0]) : nullptr;
    Trie* tr = argc >= 2 ? unwrap_external<Trie>(env, argv[1]) : nullptr;
    const uint8_t* data = nullptr;
    size_t len = 0;
    if (!ctx_usable(c) || !tr || !tr->trie || tr->destroy_pending || argc < 4 || !get_bytes(env, argv[2], &data, &len)) {
        napi_throw_type_error(env, nullptr, "encode(ctx, trie, Uint8Array, chunkSize)");
        return nullptr;
    }
    auto* w = new EncodeWork();
    w->c = c;
    ++c->refs;        // released by encode_complete
    w->trie = tr;
    ++tr->inflight;
    w->data = data;
    w->len = len;
    napi_get_value_uint32(env, argv[3], &w->cs);
    napi_value promise, name;
    NAPI_CALL(env, napi_create_promise(env, &w->deferred, &promise));
    NAPI_CALL(env, napi_create_reference(env, argv[2], 1, &w->keep_in));
    NAPI_CALL(env, napi_create_reference(env, argv[0], 1, &w->keep_ctx));
    NAPI_CALL(env, napi_create_reference(env, argv[1], 1, &w->keep_trie));
    NAPI_CALL(env, napi_create_string_utf8(env, "gpubpe.encode", NAPI_AUTO_LENGTH, &name));
    NAPI_CALL(env, napi_create_async_work(env, nullptr, name, encode_execute, encode_complete, w, &w->work));
    NAPI_CALL(env, napi_queue_async_work(env, w->work));
    return promise;
}

napi_value Init(napi_env env, napi_value exports) {
    napi_property_descriptor props[] = {
        {"createContext", nullptr, CreateContext, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"destroyContext", nullptr, DestroyContext, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"limits", nullptr, Limits, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"kernelNames", nullptr, KernelNames, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"wordBoundary", nullptr, WordBoundary, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"pretokenizeGpt4", nullptr, PretokenizeGpt4, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"trainerCreate", nullptr, TrainerCreate, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"trainerStep", nullptr, TrainerStep, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"trainerDestroy", nullptr, TrainerDestroy, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"trieUpload", nullptr, TrieUpload, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"bpeUpload", nullptr, BpeUpload, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"bpeEncode", nullptr, BpeEncode, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"trieFree", nullptr, TrieFree, nullptr, nullptr, nullptr, napi_default, nullptr},
        {"encode", nullptr, Encode, nullptr, nullptr, nullptr, napi_default, nullptr},
    };
    napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)

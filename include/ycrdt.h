/* ycrdt.h — C ABI of the MI355X-native batched Yjs merge engine (libycrdt.so).
 *
 * This is the drop-in boundary for the path @ypear/crdt delegates to Yjs. The reference injects
 * its CRDT engine through `router.options.Y` (reference crdt.js:175-180) and only ever calls the
 * entry points listed below; each function cites the reference call sites it replaces. A Node
 * N-API addon (crdt_amd/js) and a Python ctypes mirror (crdt_amd/__init__.py) are the callers.
 *
 * Conventions
 *  - Inputs are borrowed for the duration of the call and copied (to HBM) before it returns.
 *  - Outputs (ycrdt_out) are library-owned until ycrdt_free().
 *  - Every function returns YCRDT_OK (0) or a negative YCRDT_E_* code; ycrdt_last_error() gives
 *    the message (thread-local). Decode errors are atomic: the doc is unchanged (Yjs decodes the
 *    whole struct section before integrating, Y@21330).
 *  - Output byte order is Yjs 13.6 canonical (delete-set / state-vector clients sorted
 *    descending); see DESIGN.md §Compat for the 13.5.16 insertion-order difference.
 *  - There is no CPU fallback: without a usable HIP device every compute entry point fails
 *    with YCRDT_E_DEVICE.
 *  - Threads: calls on one engine are serialised by the caller, with one exception — a batch may
 *    be created (ycrdt_batch_stage*: host packing + H2D on the engine's copy stream) by one thread
 *    while another thread merges a different batch or reads its result (the serving loop:
 *    batch k+1 staged beside batch k's merge).
 */
#ifndef YCRDT_H
#define YCRDT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ycrdt_engine ycrdt_engine;
typedef struct ycrdt_doc ycrdt_doc;
typedef struct ycrdt_batch ycrdt_batch;
typedef struct ycrdt_comm ycrdt_comm; /* RCCL communicator (multi-GPU exchanges) */
#define YCRDT_COMM_ID_BYTES 128

typedef struct { const uint8_t *ptr; size_t len; } ycrdt_buf; /* borrowed */
typedef struct { uint8_t *ptr; size_t len; } ycrdt_out;       /* library-owned */

enum {
  YCRDT_OK = 0,
  YCRDT_E_DECODE = -1,      /* malformed update (Yjs: Error('Integer out of range!')) */
  YCRDT_E_PENDING = -2,     /* internal: missing dependencies seen by a merge that must have none */
  YCRDT_E_UNSUPPORTED = -3, /* valid Yjs input outside the engine's coverage */
  YCRDT_E_CAPACITY = -4,
  YCRDT_E_DEVICE = -5,      /* no HIP device / HIP runtime error */
  YCRDT_E_ARG = -6,
};

typedef struct {
  uint64_t in_bytes;        /* bytes of all input updates */
  uint64_t items;           /* Σ struct clock lengths of the inputs (Item + GC, Skip excluded) */
  uint64_t structs;         /* decoded structs */
  uint64_t units;           /* distinct (client, clock) units in the merged store */
  uint64_t segments;        /* split-point segments */
  uint64_t out_structs;     /* structs in the encoded state */
  uint64_t out_bytes;       /* encoded update bytes */
  uint64_t clients;
  double device_ms;         /* device time of the merge (events on the engine stream) */
} ycrdt_merge_stats;

/* ---- engine ------------------------------------------------------------------------------ */
/* device: HIP device ordinal. compat: 136 (default, Yjs 13.6 order) */
int ycrdt_engine_create(int device, int compat, ycrdt_engine **out);
void ycrdt_engine_destroy(ycrdt_engine *e);
/* optional per-phase device timing (hipEvents on the engine stream) */
int ycrdt_engine_set_profiling(ycrdt_engine *e, int on);
/* fills up to `cap` (name, milliseconds) pairs of the last merge; returns the count */
int ycrdt_engine_phase_times(ycrdt_engine *e, const char **names, double *ms, int cap);
/* HBM the engine holds: its grow-only merge workspace, the doc-state arena and the staging batch */
int ycrdt_engine_device_bytes(ycrdt_engine *e, uint64_t *bytes);
/* Releases the engine's merge workspace (grow-only HBM buffers) and every doc's spare state block
 * (a folded merge keeps the previous state's block for the next one; doc states and batches stay):
 * after a giant merge, e.g. the >= 1 B-item replay of crdt.js:79-98, a server gets its HBM back.
 * The next merge allocates what it needs again. */
int ycrdt_engine_trim(ycrdt_engine *e);

/* ---- Y.Doc ------------------------------------------------------------------------------- */
/* new Y.Doc()  (crdt.js:33,54,56,80,221) */
int ycrdt_doc_create(ycrdt_engine *e, uint32_t client_id, ycrdt_doc **out);
void ycrdt_doc_destroy(ycrdt_doc *d);
/* Y.applyUpdate(doc, u8)  (crdt.js:35,56,58,85,294). Yjs semantics, including missing
 * dependencies: structs whose dependencies are unknown are parked (Yjs store.pendingStructs /
 * pendingDs, readUpdateV2 Y@21330), retried when a later update supplies them, and emitted by
 * ycrdt_encode_state_as_update exactly as Yjs does. The update is validated now (a malformed one
 * fails with YCRDT_E_DECODE: the doc is unchanged if the struct section is malformed; a malformed
 * delete set keeps the structs and the ranges read before the error, as in Yjs); the merge itself
 * is DEFERRED to the next read of the doc (encode*, json, map_type_at, a local op, flush), so a
 * burst of n applies costs one batched merge (crdt.js:294 onData bursts, crdt.js:79-98 replay). */
int ycrdt_apply_update(ycrdt_doc *d, ycrdt_buf update);
/* n sequential Y.applyUpdate calls (LevelDB replay crdt.js:79-98, ingest); stops at the first
 * malformed update, as a loop of Y.applyUpdate would. */
int ycrdt_apply_updates(ycrdt_doc *d, const ycrdt_buf *ups, size_t n);
/* Fleet ingest (crdt.js:235 one doc per topic, crdt.js:294 onData per message):
 * Y.applyUpdate(docs[i], ups[i]) for i = 0..n-1, validated as ycrdt_apply_updates, then merged in
 * this call — ONE device pass for every document that has nothing pending (multi-document batch,
 * results split back into each document's HBM state on the device). Documents with pending
 * structs / delete ranges, or an engine with compat 135, take their own flush. All documents must
 * belong to `e`. A malformed update i: updates before it are applied (and merged), then
 * YCRDT_E_DECODE. */
int ycrdt_apply_updates_multi(ycrdt_engine *e, ycrdt_doc *const *docs, const ycrdt_buf *ups, size_t n);
/* Y.encodeStateAsUpdate + Y.encodeStateVector of n documents in one call (a fleet's LevelDB
 * snapshot / sync answers, crdt.js:33-40,260,288): deferred applies are flushed as one batched merge
 * and the states gathered on the device, then copied with one pipelined D2H. Document i's update
 * is dst[offs[2i] .. offs[2i+1]), its state vector dst[offs[2i+1] .. offs[2i+2]); offs holds 2n+1
 * entries. dst == NULL only fills offs / total (size query). */
int ycrdt_docs_states_packed(ycrdt_engine *e, ycrdt_doc *const *docs, size_t n, uint8_t *dst, uint64_t cap, uint64_t *offs,
                             uint64_t *total);
/* Runs the deferred applies now (every read does this implicitly). */
int ycrdt_doc_flush(ycrdt_doc *d);
/* Whether Yjs would hold pending structs (store.pendingStructs) / a pending delete set
 * (store.pendingDs) for this doc. */
int ycrdt_doc_pending(ycrdt_doc *d, int *structs, int *delete_set);
/* Y.encodeStateAsUpdate(doc[, sv])  (crdt.js:56,260,288,347,383,443,471,505,533,560,585,611);
 * sv.len == 0 ⇒ full state */
int ycrdt_encode_state_as_update(ycrdt_doc *d, ycrdt_buf sv, ycrdt_out *out);
/* Y.encodeStateVector(doc)  (crdt.js:59,239,258,289) */
int ycrdt_encode_state_vector(ycrdt_doc *d, ycrdt_out *out);
/* stats of the doc's last merge */
int ycrdt_doc_last_stats(ycrdt_doc *d, ycrdt_merge_stats *st);

/* Y.mergeUpdates(updates) — north_star; Yjs-internal for pending structs (Y@39011). Lazy k-way
 * merge of the updates' structs (no integration), delete sets unioned. One input is returned
 * unchanged, as Yjs does. */
int ycrdt_merge_updates(ycrdt_engine *e, const ycrdt_buf *ups, size_t n, ycrdt_out *out);
/* Y.diffUpdate(update, sv) (Y@40711): the structs of `update` missing from state vector `sv`,
 * with the update's delete set. */
int ycrdt_diff_update(ycrdt_engine *e, ycrdt_buf update, ycrdt_buf sv, ycrdt_out *out);
/* n independent Y.diffUpdate(updates[i], svs[i]) in ONE batched device pass: the sync responder
 * of crdt.js:286-291 (`Y.encodeStateAsUpdate(doc, peerStateVector)` per joining peer) batched
 * across peers and topics. outs[i] is byte-identical to
 * ycrdt_diff_update(updates[i], svs[i]); each must be released with ycrdt_free. A malformed
 * update or state vector fails the whole batch (no output is produced). */
int ycrdt_diff_updates(ycrdt_engine *e, const ycrdt_buf *updates, const ycrdt_buf *svs, size_t n, ycrdt_out *outs);

/* ---- crdt.c materialisation and local ops ------------------------------------------------
 * A "target" is root type `root`, or (parent_key != NULL) the shared type stored in root YMap
 * `root` under `parent_key` (crdt.js nests one YArray per map key, crdt.js:423-430).
 * The device computes map winners and list order (a view of the merged state); the host
 * decodes values and writes each local op as a one-struct Yjs v1 update, applied like a remote
 * one, so the doc's bytes match a Yjs doc that performed the same ops. */
/* YMap.toJSON / YArray.toJSON of a root (kind 0 = map, 1 = array) as JSON.stringify text
 * (crdt.js:202,214,304,372,494,528,555,581,607; YMap.toJSON Y@51558, typeListToArray Y@46408) */
int ycrdt_doc_json(ycrdt_doc *d, const char *root, int kind, ycrdt_out *out);
/* toJSON of the shared type at a target (parent_key == NULL: root type `root`; else the YMap
 * (kind 0) / YArray (kind 1) stored in root map `root` under parent_key — crdt.js:423-430 nests one
 * YArray per key): reads that type's own list only. A key holding no such type gives {} / []. */
int ycrdt_type_json(ycrdt_doc *d, const char *root, const char *parent_key, int kind, ycrdt_out *out);
/* The live entries of a YMap target with the id of each entry's winning item, as JSON text
 * {"key": ["client:clock", value], ...} — what YMap.observe's keysChanged (Y@51190) is computed
 * from: a key changed iff its winning item changed (crdt.js:620-657 observers). */
int ycrdt_map_entries(ycrdt_doc *d, const char *root, const char *parent_key, ycrdt_out *out);
/* YMap.get(key) of root map `root`: *type_ref = the type ref (0 YArray, 1 YMap, ...) when the
 * key holds a live shared type, else -1 (a plain value or nothing)  (crdt.js:423-424) */
int ycrdt_map_type_at(ycrdt_doc *d, const char *root, const char *key, int32_t *type_ref);
/* YMap.set(key, value) with a lib0 `any` value (crdt.js:375,434; typeMapSet Y@49334) */
int ycrdt_map_set(ycrdt_doc *d, const char *root, const char *parent_key, const char *key, const uint8_t *any,
                  size_t anylen);
/* YMap.set(key, new Y.Array()) (type_ref 0) / new Y.Map() (1)  (crdt.js:423) */
int ycrdt_map_set_type(ycrdt_doc *d, const char *root, const char *parent_key, const char *key, uint32_t type_ref);
/* YMap.delete(key)  (crdt.js:465; typeMapDelete Y@49261) */
int ycrdt_map_delete(ycrdt_doc *d, const char *root, const char *parent_key, const char *key);
/* YArray.insert(index, values) / push / unshift with `count` concatenated lib0 `any` values
 * (crdt.js:426-428,527,554,580; typeListInsertGenerics Y@48365). "Length exceeded!" past the end. */
int ycrdt_array_insert(ycrdt_doc *d, const char *root, const char *parent_key, uint32_t index, const uint8_t *anys,
                       size_t len, uint32_t count);
/* YArray.delete(index, length)  (crdt.js:429,606; typeListDelete Y@48835). Like Yjs, deletes
 * what exists and then fails with "Length exceeded!" when the range runs past the end. */
int ycrdt_array_delete(ycrdt_doc *d, const char *root, const char *parent_key, uint32_t index, uint32_t length);
/* doc.clientID */
int ycrdt_doc_client_id(ycrdt_doc *d, uint32_t *out);
/* Per-key reads of the materialised view, replacing a full toJSON per call (facade YMap.get / has /
 * size, YArray.length / get; crdt.js:423-424 `h[name].has(key)` / `.get(key)`, push's length):
 * state 0 = absent, 1 = present (`json` = JSON text of the value), 2 = present, value `undefined`.
 * `json` is always allocated (free with ycrdt_free). A nested target whose type does not exist
 * reads as empty. */
int ycrdt_map_get(ycrdt_doc *d, const char *root, const char *parent_key, const char *key, int *state, ycrdt_out *json);
int ycrdt_map_size(ycrdt_doc *d, const char *root, const char *parent_key, uint32_t *size);
int ycrdt_array_length(ycrdt_doc *d, const char *root, const char *parent_key, uint64_t *length);
int ycrdt_array_get(ycrdt_doc *d, const char *root, const char *parent_key, uint64_t index, int *state, ycrdt_out *json);
/* Incremental local-op encode: the updates of the local ops
 * (ycrdt_map_* / ycrdt_array_*) applied since the previous call, as ONE update (Y.mergeUpdates of
 * them; a single op's own update is returned as is; none = the empty update). crdt.js broadcasts
 * Y.encodeStateAsUpdate(doc) after every local op (crdt.js:347,383,443,471,505,533,560,585,611);
 * this delta is wire-compatible (Y.applyUpdate accepts it) but changes the bytes on the wire, so a
 * host opts in. Remote updates applied in between are not part of it. */
int ycrdt_doc_take_local_update(ycrdt_doc *d, ycrdt_out *out);
/* Starts (on != 0) or stops recording local-op updates for ycrdt_doc_take_local_update. Off by
 * default; the first take turns it on. A long untaken list is folded into one update. */
int ycrdt_doc_track_local(ycrdt_doc *d, int on);

/* ---- device-resident batches (ingest queue / benchmark) ---------------------------------- */
/* Copies the updates into HBM. */
int ycrdt_batch_stage(ycrdt_engine *e, const ycrdt_buf *ups, size_t n, ycrdt_batch **out);
/* Merges the staged updates into a fresh doc entirely on the device; the encoded state stays in
 * HBM. Equivalent to applying every update to a new Y.Doc and encodeStateAsUpdate(doc). */
int ycrdt_batch_merge(ycrdt_batch *b, ycrdt_merge_stats *st);
/* Copies the merge result (encoded update and state vector) to the host. The result lives in the
 * engine workspace: any other engine call in between makes this fail with YCRDT_E_ARG. */
int ycrdt_batch_result(ycrdt_batch *b, ycrdt_out *update, ycrdt_out *state_vector);
void ycrdt_batch_destroy(ycrdt_batch *b);
/* Multi-document batches (C5 fleets: one Y.Doc per topic, crdt.js:235; and many independent replica
 * sets per device pass): update i belongs to document doc_of[i] < ndocs. One device pass merges
 * every document on its own (clients, lists and delete sets never mix across documents); the
 * result of document d equals merging its updates alone. */
int ycrdt_batch_stage_docs(ycrdt_engine *e, const ycrdt_buf *ups, const uint32_t *doc_of, size_t n, uint32_t ndocs,
                           ycrdt_batch **out);
/* updates[ndocs] (and state_vectors[ndocs] unless NULL) receive every document's encoded state */
int ycrdt_batch_result_docs(ycrdt_batch *b, ycrdt_out *updates, ycrdt_out *state_vectors);
/* The same results packed back to back in caller memory, split per document on the device (one
 * HBM buffer, one pipelined D2H through pinned staging; no per-document allocation): document d's
 * encodeStateAsUpdate is dst[offs[2d] .. offs[2d+1]) and its encodeStateVector dst[offs[2d+1] ..
 * offs[2d+2]); offs holds 2*ndocs+1 entries, *total = offs[2*ndocs]. dst == NULL only fills offs /
 * total (size query); cap < total is YCRDT_E_ARG. A sync responder / LevelDB writer hands the
 * slices on as they are (crdt.js:260,288 send Y.encodeStateAsUpdate bytes; crdt.js:79-98 store). */
int ycrdt_batch_result_docs_packed(ycrdt_batch *b, uint8_t *dst, uint64_t cap, uint64_t *offs, uint64_t *total);
/* one-shot form of the two above (host buffers in and out) */
int ycrdt_merge_docs(ycrdt_engine *e, const ycrdt_buf *ups, const uint32_t *doc_of, size_t n, uint32_t ndocs,
                     ycrdt_out *updates, ycrdt_out *state_vectors);

/* ---- host-only entry points (no HIP device needed) ---------------------------------------- */
/* The validation Y.applyUpdate runs before queueing an update: YCRDT_OK, or YCRDT_E_DECODE with
 * *structs_ok = 1 when only the delete set is malformed (Yjs then keeps the structs). */
int ycrdt_validate_update(ycrdt_buf update, int *structs_ok);
/* Test hook for the pending-struct emulation (yc_ingest.cpp): replays n Y.applyUpdate calls into
 * an empty doc on struct headers only, with Y.mergeUpdates supplied by the caller (`merge` fills
 * *out with caller-owned bytes that must stay valid until it returns). Outputs the store's state
 * vector (clients ascending), the pending-structs update (len 0 = none) and the pending delete set
 * (len 0 = none); release them with ycrdt_free. */
typedef int (*ycrdt_merge_fn)(void *ctx, const ycrdt_buf *ups, size_t n, ycrdt_out *out);
int ycrdt_debug_replay(const ycrdt_buf *ups, size_t n, ycrdt_merge_fn merge, void *ctx, ycrdt_out *sv,
                       ycrdt_out *pending, ycrdt_out *pending_ds);

/* ---- multi-GPU: RCCL over xGMI inside the library, one rank per GPU.
 * Rank 0 creates the unique id; the caller hands those bytes to every rank (any channel), then each
 * rank creates its communicator on its engine's device. */
int ycrdt_comm_unique_id(uint8_t id[YCRDT_COMM_ID_BYTES]);
int ycrdt_comm_create(ycrdt_engine *e, int nranks, int rank, const uint8_t id[YCRDT_COMM_ID_BYTES], ycrdt_comm **out);
void ycrdt_comm_destroy(ycrdt_comm *c);
/* A communicator over the caller's own transport: the library's exchanges run their collectives
 * through these host callbacks instead of RCCL (device buffers are staged through host memory).
 * Each callback returns 0 on success; every rank must make the same calls in the same order. Used
 * by hosts without RCCL between their processes (and by the world-size-2 gloo tests, two processes
 * on one GPU). Failure inside an exchange: a rank that fails between two collectives of one
 * exchange cannot abort a host transport the way it aborts an RCCL communicator (ncclCommAbort),
 * so its peers stay in the callback they are in until the TRANSPORT gives up: host transports must
 * carry their own timeout (gloo's process-group timeout does) and return nonzero from the callback,
 * which then fails the merge on that rank. Failures before an exchange never block: every exchange
 * starts with a one-word status agreement. */
typedef struct {
  void *ctx;
  /* in place over n host words of every rank: op 0 = sum, 1 = max */
  int (*allreduce_u32)(void *ctx, uint32_t *words, size_t n, int op);
  /* recv[r * bytes .. (r + 1) * bytes) = rank r's send (bytes is the same on every rank) */
  int (*allgather)(void *ctx, const uint8_t *send, size_t bytes, uint8_t *recv);
} ycrdt_exchange;
int ycrdt_comm_create_exchange(ycrdt_engine *e, int nranks, int rank, const ycrdt_exchange *x, ycrdt_comm **out);
/* Stable owner rank of a document / topic id (crdt.js:221,235: one Y.Doc per topic): the same on
 * every rank, process and run (64-bit FNV-1a of the id bytes, mixed, mod world). A fleet routes
 * every update of a topic to its owner, which merges it alone (weak scaling, no data collective). */
uint32_t ycrdt_route(const uint8_t *id, size_t len, uint32_t world);
/* Key-hash sharded merge of ONE document (C4): every rank stages the same updates; the integrate
 * phases (map winner, YATA, dead types, merge adjacency) run for the rank's shard only — lists
 * owned by hash(top-level entry) % nshards — and the per-segment flag words are summed over RCCL;
 * every rank then encodes the full result. comm == NULL: all nshards logical shards run in turn on
 * this GPU (the partition check: byte-identical to ycrdt_batch_merge). Read the result with
 * ycrdt_batch_result. */
int ycrdt_batch_merge_sharded(ycrdt_batch *b, ycrdt_comm *comm, uint32_t nshards, ycrdt_merge_stats *st);
/* State vector of the union of what the ranks hold of one document (crdt.js:239,289 exchange):
 * all-gather + max per client, descending client order. */
int ycrdt_comm_sv_allreduce_max(ycrdt_comm *c, ycrdt_engine *e, ycrdt_buf sv, ycrdt_out *out);
/* Fleet state vectors (C5; crdt.js:239,289 per topic, batched over the fleet): this rank holds n
 * documents (ids docs[i] < 0xFFFFFFFF, state vectors svs[i]) — any subset of the fleet. Every rank
 * receives, for each document ANY rank holds, the state vector of the union (max clock per client,
 * descending client order): *doc_ids = u32[m] ascending, *offs = u64[m + 1], document doc_ids[j]'s
 * state vector = blob[offs[j] .. offs[j+1]). One dense all-reduce(MAX) over the fleet's sorted
 * (document, client) key space, built on the device (sort, reduce, all-gather of distinct keys,
 * unique). Release the three outputs with ycrdt_free. */
int ycrdt_comm_fleet_sv_allreduce_max(ycrdt_comm *c, ycrdt_engine *e, const uint32_t *docs, const ycrdt_buf *svs, size_t n,
                                      ycrdt_out *doc_ids, ycrdt_out *offs, ycrdt_out *blob);
/* Delete sets of all ranks (each a delete-set-only or full update) all-gathered and merged with the
 * engine's HIP mergeUpdates (the delete-set union): every rank receives the same update. */
int ycrdt_comm_ds_allgather(ycrdt_comm *c, ycrdt_engine *e, ycrdt_buf update, ycrdt_out *out);

/* Every rank's byte string, in rank order (variable lengths): blob = the concatenation, offs =
 * (nranks + 1) u64 offsets into it. The host-side control exchange of a multi-rank job (barrier,
 * the max of the ranks' step times, per-rank reports) over the library's own transport. */
int ycrdt_comm_allgather(ycrdt_comm *c, ycrdt_engine *e, ycrdt_buf mine, ycrdt_out *blob, ycrdt_out *offs);
/* HIP devices visible to this process (a launcher assigns rank r to device r % count) */
int ycrdt_device_count(int *count);

void ycrdt_free(ycrdt_out *o);
const char *ycrdt_last_error(void);
const char *ycrdt_version(void);

#ifdef __cplusplus
}
#endif
#endif

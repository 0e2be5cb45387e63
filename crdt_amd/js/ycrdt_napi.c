/* ycrdt_napi.c — Node-API addon over the C ABI (include/ycrdt.h).
 *
 * This is the reference-language host binding: @ypear/crdt loads its CRDT engine from
 * `router.options.Y` (reference crdt.js:175-180), so a Node module exporting the Yjs functions
 * the reference calls is the drop-in. crdt_amd/js/index.js builds that `Y` object on top of this
 * binding. Plain C + node_api.h (NAPI 8, Node >= 12.22); no node-gyp needed:
 *   gcc -shared -fPIC -I/usr/include/node ycrdt_napi.c -L.. -lycrdt -Wl,-rpath,'$ORIGIN/..'
 * Errors from the engine become JS `Error`s carrying ycrdt_last_error() (the reference only reads
 * e.message, crdt.js:38-39) and a numeric `code`.
 */
#define NAPI_VERSION 8
#include <node_api.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/ycrdt.h"

#define CHECK(env, call)                                                 \
  do {                                                                   \
    if ((call) != napi_ok) {                                             \
      napi_throw_error((env), NULL, "ycrdt: N-API call failed: " #call); \
      return NULL;                                                       \
    }                                                                    \
  } while (0)

static ycrdt_engine *g_engine = NULL; /* one engine (HIP device + stream) per process */
static int g_device = 0;

static napi_value throw_rc(napi_env env, int rc) {
  napi_value msg, err, code;
  const char *m = ycrdt_last_error();
  napi_create_string_utf8(env, m && m[0] ? m : "ycrdt error", NAPI_AUTO_LENGTH, &msg);
  napi_create_error(env, NULL, msg, &err);
  napi_create_int32(env, rc, &code);
  napi_set_named_property(env, err, "code", code);
  napi_throw(env, err);
  return NULL;
}

static ycrdt_engine *engine(napi_env env) {
  if (!g_engine) {
    /* YCRDT_COMPAT=135: Yjs 13.5.16 client order in delete sets / state vectors (include/ycrdt.h) */
    const char *cv = getenv("YCRDT_COMPAT");
    int rc = ycrdt_engine_create(g_device, cv && atoi(cv) == 135 ? 135 : 136, &g_engine);
    if (rc != YCRDT_OK) {
      g_engine = NULL;
      throw_rc(env, rc);
      return NULL;
    }
  }
  return g_engine;
}

/* Uint8Array / Buffer argument → borrowed (ptr, len) */
static int get_bytes(napi_env env, napi_value v, ycrdt_buf *out) {
  bool is_ta = false;
  napi_is_typedarray(env, v, &is_ta);
  if (is_ta) {
    napi_typedarray_type t;
    size_t len, off;
    void *data;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &t, &len, &data, &ab, &off) != napi_ok || t != napi_uint8_array) return 0;
    out->ptr = (const uint8_t *)data;
    out->len = len;
    return 1;
  }
  bool is_buf = false;
  napi_is_buffer(env, v, &is_buf);
  if (is_buf) {
    void *data;
    size_t len;
    if (napi_get_buffer_info(env, v, &data, &len) != napi_ok) return 0;
    out->ptr = (const uint8_t *)data;
    out->len = len;
    return 1;
  }
  return 0;
}


static napi_value u8_from_out(napi_env env, ycrdt_out *o) {
  napi_value ab, ta;
  void *data = NULL;
  size_t n = o->len;
  CHECK(env, napi_create_arraybuffer(env, n, &data, &ab));
  if (n) memcpy(data, o->ptr, n);
  ycrdt_free(o);
  CHECK(env, napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &ta));
  return ta;
}

static void doc_finalize(napi_env env, void *data, void *hint) {
  (void)env;
  (void)hint;
  ycrdt_doc_destroy((ycrdt_doc *)data);
}

static ycrdt_doc *get_doc(napi_env env, napi_value v) {
  void *p = NULL;
  if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
    napi_throw_type_error(env, NULL, "ycrdt: expected a doc handle");
    return NULL;
  }
  return (ycrdt_doc *)p;
}

/* setDevice(ordinal) — before the first engine use */
static napi_value js_set_device(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int32_t dev = 0;
  if (argc > 0) napi_get_value_int32(env, argv[0], &dev);
  g_device = dev;
  return NULL;
}

/* docCreate(clientId) → handle   (new Y.Doc(), crdt.js:33,54,56,80,221) */
static napi_value js_doc_create(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], out;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  uint32_t cid = 0;
  if (argc > 0) napi_get_value_uint32(env, argv[0], &cid);
  ycrdt_engine *e = engine(env);
  if (!e) return NULL;
  ycrdt_doc *d = NULL;
  int rc = ycrdt_doc_create(e, cid, &d);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  CHECK(env, napi_create_external(env, d, doc_finalize, NULL, &out));
  return out;
}

/* applyUpdates(doc, update | update[])   (Y.applyUpdate, crdt.js:35,56,58,85,294) */
static napi_value js_apply_updates(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 2) { napi_throw_type_error(env, NULL, "applyUpdates(doc, updates)"); return NULL; }
  ycrdt_doc *d = get_doc(env, argv[0]);
  if (!d) return NULL;
  bool is_arr = false;
  napi_is_array(env, argv[1], &is_arr);
  if (!is_arr) {
    ycrdt_buf b;
    if (!get_bytes(env, argv[1], &b)) { napi_throw_type_error(env, NULL, "update must be a Uint8Array"); return NULL; }
    int rc = ycrdt_apply_update(d, b);
    return rc == YCRDT_OK ? NULL : throw_rc(env, rc);
  }
  uint32_t n = 0;
  napi_get_array_length(env, argv[1], &n);
  ycrdt_buf *bufs = (ycrdt_buf *)calloc(n ? n : 1, sizeof(ycrdt_buf));
  for (uint32_t i = 0; i < n; ++i) {
    napi_value el;
    napi_get_element(env, argv[1], i, &el);
    if (!get_bytes(env, el, &bufs[i])) {
      free(bufs);
      napi_throw_type_error(env, NULL, "updates must be Uint8Arrays");
      return NULL;
    }
  }
  int rc = ycrdt_apply_updates(d, bufs, n);
  free(bufs);
  return rc == YCRDT_OK ? NULL : throw_rc(env, rc);
}

/* encodeStateAsUpdate(doc[, sv])   (crdt.js:56,260,288,347,383,443,471,505,533,560,585,611) */
/* applyUpdatesMulti(docs[], updates[]) — Y.applyUpdate(docs[i], updates[i]) for a fleet, merged in
 * one device pass (ycrdt_apply_updates_multi; crdt.js:235 one doc per topic, :294 onData) */
static napi_value js_apply_updates_multi(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bool a0 = false, a1 = false;
  if (argc >= 2) { napi_is_array(env, argv[0], &a0); napi_is_array(env, argv[1], &a1); }
  uint32_t n = 0, m = 0;
  if (a0) napi_get_array_length(env, argv[0], &n);
  if (a1) napi_get_array_length(env, argv[1], &m);
  if (!a0 || !a1 || n != m) { napi_throw_type_error(env, NULL, "applyUpdatesMulti(docs[], updates[]) of equal length"); return NULL; }
  ycrdt_engine *e = engine(env);
  if (!e) return NULL;
  ycrdt_doc **docs = (ycrdt_doc **)calloc(n ? n : 1, sizeof(ycrdt_doc *));
  ycrdt_buf *bufs = (ycrdt_buf *)calloc(n ? n : 1, sizeof(ycrdt_buf));
  if (!docs || !bufs) {
    free(docs); free(bufs);
    napi_throw_error(env, NULL, "applyUpdatesMulti: out of host memory");
    return NULL;
  }
  for (uint32_t i = 0; i < n; ++i) {
    napi_value d, u;
    napi_get_element(env, argv[0], i, &d);
    napi_get_element(env, argv[1], i, &u);
    docs[i] = get_doc(env, d);
    /* get_doc has already thrown for a non-Doc; only a bad update still needs an error */
    const int doc_ok = docs[i] != NULL;
    if (!doc_ok || !get_bytes(env, u, &bufs[i])) {
      free(docs); free(bufs);
      if (doc_ok) napi_throw_type_error(env, NULL, "updates must be Uint8Arrays");
      return NULL;
    }
  }
  int rc = ycrdt_apply_updates_multi(e, docs, bufs, n);
  free(docs); free(bufs);
  return rc == YCRDT_OK ? NULL : throw_rc(env, rc);
}

static napi_value js_encode_state_as_update(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ycrdt_doc *d = argc > 0 ? get_doc(env, argv[0]) : NULL;
  if (!d) return NULL;
  ycrdt_buf sv = {NULL, 0};
  if (argc > 1) {
    napi_valuetype t;
    napi_typeof(env, argv[1], &t);
    if (t != napi_undefined && t != napi_null && !get_bytes(env, argv[1], &sv)) {
      napi_throw_type_error(env, NULL, "state vector must be a Uint8Array");
      return NULL;
    }
  }
  ycrdt_out o = {NULL, 0};
  int rc = ycrdt_encode_state_as_update(d, sv, &o);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  return u8_from_out(env, &o);
}

/* encodeStateVector(doc)   (crdt.js:59,239,258,289) */
static napi_value js_encode_state_vector(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ycrdt_doc *d = argc > 0 ? get_doc(env, argv[0]) : NULL;
  if (!d) return NULL;
  ycrdt_out o = {NULL, 0};
  int rc = ycrdt_encode_state_vector(d, &o);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  return u8_from_out(env, &o);
}

/* takeLocalUpdate(doc) → Uint8Array: the local ops since the previous call as one update */
static napi_value js_take_local_update(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ycrdt_doc *d = argc > 0 ? get_doc(env, argv[0]) : NULL;
  if (!d) return NULL;
  ycrdt_out o = {NULL, 0};
  int rc = ycrdt_doc_take_local_update(d, &o);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  return u8_from_out(env, &o);
}

/* trackLocalUpdates(doc[, on = true]): record local-op updates for takeLocalUpdate (opt-in) */
static napi_value js_track_local(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ycrdt_doc *d = argc > 0 ? get_doc(env, argv[0]) : NULL;
  if (!d) return NULL;
  bool on = true;
  if (argc > 1) CHECK(env, napi_get_value_bool(env, argv[1], &on));
  int rc = ycrdt_doc_track_local(d, on ? 1 : 0);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  return NULL;
}

/* lastStats(doc) → {items, structs, units, segments, outBytes, deviceMs} */
static napi_value js_last_stats(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], obj, v;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ycrdt_doc *d = argc > 0 ? get_doc(env, argv[0]) : NULL;
  if (!d) return NULL;
  ycrdt_merge_stats st;
  int rc = ycrdt_doc_last_stats(d, &st);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  CHECK(env, napi_create_object(env, &obj));
#define PUT(name, val) napi_create_double(env, (double)(val), &v); napi_set_named_property(env, obj, name, v)
  PUT("inBytes", st.in_bytes);
  PUT("items", st.items);
  PUT("structs", st.structs);
  PUT("units", st.units);
  PUT("segments", st.segments);
  PUT("outBytes", st.out_bytes);
  PUT("clients", st.clients);
  PUT("deviceMs", st.device_ms);
#undef PUT
  return obj;
}

/* mergeUpdates(update[]) → Uint8Array   (Y.mergeUpdates, north_star / Y@39011) */
static napi_value js_merge_updates(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  bool is_arr = false;
  if (argc > 0) napi_is_array(env, argv[0], &is_arr);
  if (!is_arr) { napi_throw_type_error(env, NULL, "mergeUpdates(updates[])"); return NULL; }
  ycrdt_engine *e = engine(env);
  if (!e) return NULL;
  uint32_t n = 0;
  napi_get_array_length(env, argv[0], &n);
  ycrdt_buf *bufs = (ycrdt_buf *)calloc(n ? n : 1, sizeof(ycrdt_buf));
  for (uint32_t i = 0; i < n; ++i) {
    napi_value el;
    napi_get_element(env, argv[0], i, &el);
    if (!get_bytes(env, el, &bufs[i])) { free(bufs); napi_throw_type_error(env, NULL, "updates must be Uint8Arrays"); return NULL; }
  }
  ycrdt_out o = {NULL, 0};
  int rc = ycrdt_merge_updates(e, bufs, n, &o);
  free(bufs);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  return u8_from_out(env, &o);
}

/* diffUpdate(update, sv) → Uint8Array   (Y.diffUpdate, Y@40711) */
static napi_value js_diff_update(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ycrdt_buf u, sv;
  if (argc < 2 || !get_bytes(env, argv[0], &u) || !get_bytes(env, argv[1], &sv)) {
    napi_throw_type_error(env, NULL, "diffUpdate(update, stateVector)");
    return NULL;
  }
  ycrdt_engine *e = engine(env);
  if (!e) return NULL;
  ycrdt_out o = {NULL, 0};
  int rc = ycrdt_diff_update(e, u, sv, &o);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  return u8_from_out(env, &o);
}

/* diffUpdates(update[], sv[]) → Uint8Array[]   (n x Y.diffUpdate in one batched device pass: the
 * sync responder of crdt.js:286-291 across peers / topics) */
static int get_buf_array(napi_env env, napi_value arr, ycrdt_buf **out, uint32_t *n) {
  bool is_arr = false;
  napi_is_array(env, arr, &is_arr);
  if (!is_arr) return 0;
  napi_get_array_length(env, arr, n);
  *out = (ycrdt_buf *)calloc(*n ? *n : 1, sizeof(ycrdt_buf));
  for (uint32_t i = 0; i < *n; ++i) {
    napi_value el;
    napi_get_element(env, arr, i, &el);
    if (!get_bytes(env, el, &(*out)[i])) { free(*out); *out = NULL; return 0; }
  }
  return 1;
}
static napi_value js_diff_updates(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ycrdt_buf *ups = NULL, *svs = NULL;
  uint32_t n = 0, m = 0;
  if (argc < 2 || !get_buf_array(env, argv[0], &ups, &n) || !get_buf_array(env, argv[1], &svs, &m) || n != m) {
    free(ups);
    free(svs);
    napi_throw_type_error(env, NULL, "diffUpdates(updates[], stateVectors[]) with one state vector per update");
    return NULL;
  }
  ycrdt_engine *e = engine(env);
  if (!e) { free(ups); free(svs); return NULL; }
  ycrdt_out *outs = (ycrdt_out *)calloc(n ? n : 1, sizeof(ycrdt_out));
  int rc = ycrdt_diff_updates(e, ups, svs, n, outs);
  free(ups);
  free(svs);
  if (rc != YCRDT_OK) { free(outs); return throw_rc(env, rc); }
  napi_value arr;
  napi_create_array_with_length(env, n, &arr);
  for (uint32_t i = 0; i < n; ++i) napi_set_element(env, arr, i, u8_from_out(env, &outs[i]));
  free(outs);
  return arr;
}

static napi_value js_version(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value s;
  CHECK(env, napi_create_string_utf8(env, ycrdt_version(), NAPI_AUTO_LENGTH, &s));
  return s;
}

/* ---- crdt.c materialisation and local ops (YMap / YArray methods of the facade) ------------ */
/* JS string (or null/undefined → NULL when `opt`) into a malloc'd UTF-8 buffer; 0 on a type error */
static int get_str(napi_env env, napi_value v, char **out, int opt) {
  napi_valuetype t;
  napi_typeof(env, v, &t);
  *out = NULL;
  if (opt && (t == napi_undefined || t == napi_null)) return 1;
  if (t != napi_string) return 0;
  size_t n = 0;
  if (napi_get_value_string_utf8(env, v, NULL, 0, &n) != napi_ok) return 0;
  *out = (char *)malloc(n + 1);
  if (napi_get_value_string_utf8(env, v, *out, n + 1, &n) != napi_ok) { free(*out); *out = NULL; return 0; }
  return 1;
}

typedef struct { ycrdt_doc *d; char *root, *pkey, *key; } op_args;

/* (doc, root, parentKey|null[, key]) — the target of every view/local-op call */
static int op_target(napi_env env, napi_value *argv, size_t argc, int want_key, op_args *a) {
  memset(a, 0, sizeof(*a));
  if (argc < (size_t)(3 + want_key)) { napi_throw_type_error(env, NULL, "ycrdt: missing arguments"); return 0; }
  a->d = get_doc(env, argv[0]);
  if (!a->d) return 0;
  if (!get_str(env, argv[1], &a->root, 0) || !get_str(env, argv[2], &a->pkey, 1) ||
      (want_key && !get_str(env, argv[3], &a->key, 0))) {
    free(a->root); free(a->pkey);
    napi_throw_type_error(env, NULL, "ycrdt: type name and keys must be strings");
    return 0;
  }
  return 1;
}
static void op_free(op_args *a) { free(a->root); free(a->pkey); free(a->key); }

/* docJson(doc, root, kind) → JSON text of YMap.toJSON (kind 0) / YArray.toJSON (kind 1)
 * (crdt.js:202,214,304,372,494,528,555,581,607) */
static napi_value js_doc_json(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3], s;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  ycrdt_doc *d = argc > 2 ? get_doc(env, argv[0]) : NULL;
  if (!d) return NULL;
  char *root = NULL;
  int32_t kind = 0;
  if (!get_str(env, argv[1], &root, 0) || napi_get_value_int32(env, argv[2], &kind) != napi_ok) {
    free(root);
    napi_throw_type_error(env, NULL, "docJson(doc, root, kind)");
    return NULL;
  }
  ycrdt_out o = {NULL, 0};
  int rc = ycrdt_doc_json(d, root, kind, &o);
  free(root);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  CHECK(env, napi_create_string_utf8(env, (const char *)o.ptr, o.len, &s));
  ycrdt_free(&o);
  return s;
}

/* typeJson(doc, root, parentKey, kind) → toJSON of the root type (parentKey null) or of the YMap
 * (kind 0) / YArray (kind 1) stored under root[parentKey], reading that type's own list only */
static napi_value js_type_json(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4], s;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  op_args a;
  if (!op_target(env, argv, argc, 0, &a)) return NULL;
  int32_t kind = 0;
  if (argc < 4 || napi_get_value_int32(env, argv[3], &kind) != napi_ok) {
    op_free(&a);
    napi_throw_type_error(env, NULL, "typeJson(doc, root, parentKey, kind)");
    return NULL;
  }
  ycrdt_out o = {NULL, 0};
  int rc = ycrdt_type_json(a.d, a.root, a.pkey, kind, &o);
  op_free(&a);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  CHECK(env, napi_create_string_utf8(env, (const char *)o.ptr, o.len, &s));
  ycrdt_free(&o);
  return s;
}

/* mapEntries(doc, root, parentKey) → JSON text {"key": ["client:clock", value]} (map observers) */
static napi_value js_map_entries(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3], s;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  op_args a;
  if (!op_target(env, argv, argc, 0, &a)) return NULL;
  ycrdt_out o = {NULL, 0};
  int rc = ycrdt_map_entries(a.d, a.root, a.pkey, &o);
  op_free(&a);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  CHECK(env, napi_create_string_utf8(env, o.ptr ? (const char *)o.ptr : "{}", o.ptr ? o.len : 2, &s));
  ycrdt_free(&o);
  return s;
}

/* mapSet(doc, root, parentKey, key, anyBytes)   (YMap.set, crdt.js:375,434) */
static napi_value js_map_set(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  op_args a;
  if (!op_target(env, argv, argc, 1, &a)) return NULL;
  ycrdt_buf v;
  int rc = YCRDT_E_ARG;
  if (argc > 4 && get_bytes(env, argv[4], &v)) rc = ycrdt_map_set(a.d, a.root, a.pkey, a.key, v.ptr, v.len);
  else { op_free(&a); napi_throw_type_error(env, NULL, "mapSet: value must be lib0 any bytes"); return NULL; }
  op_free(&a);
  return rc == YCRDT_OK ? NULL : throw_rc(env, rc);
}

/* mapSetType(doc, root, parentKey, key, typeRef)   (YMap.set(key, new Y.Array()), crdt.js:423) */
static napi_value js_map_set_type(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  op_args a;
  if (!op_target(env, argv, argc, 1, &a)) return NULL;
  uint32_t tr = 0;
  if (argc > 4) napi_get_value_uint32(env, argv[4], &tr);
  int rc = ycrdt_map_set_type(a.d, a.root, a.pkey, a.key, tr);
  op_free(&a);
  return rc == YCRDT_OK ? NULL : throw_rc(env, rc);
}

/* mapDelete(doc, root, parentKey, key)   (YMap.delete, crdt.js:465) */
static napi_value js_map_delete(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  op_args a;
  if (!op_target(env, argv, argc, 1, &a)) return NULL;
  int rc = ycrdt_map_delete(a.d, a.root, a.pkey, a.key);
  op_free(&a);
  return rc == YCRDT_OK ? NULL : throw_rc(env, rc);
}

/* arrayInsert(doc, root, parentKey, index, anysBytes, count)   (insert/push/unshift, crdt.js:426-428,527,554,580) */
static napi_value js_array_insert(napi_env env, napi_callback_info info) {
  size_t argc = 6;
  napi_value argv[6];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  op_args a;
  if (!op_target(env, argv, argc, 0, &a)) return NULL;
  uint32_t index = 0, count = 0;
  ycrdt_buf v;
  if (argc < 6 || napi_get_value_uint32(env, argv[3], &index) != napi_ok || !get_bytes(env, argv[4], &v) ||
      napi_get_value_uint32(env, argv[5], &count) != napi_ok) {
    op_free(&a);
    napi_throw_type_error(env, NULL, "arrayInsert(doc, root, parentKey, index, anys, count)");
    return NULL;
  }
  int rc = ycrdt_array_insert(a.d, a.root, a.pkey, index, v.ptr, v.len, count);
  op_free(&a);
  return rc == YCRDT_OK ? NULL : throw_rc(env, rc);
}

/* arrayDelete(doc, root, parentKey, index, length)   (YArray.delete, crdt.js:429,606) */
static napi_value js_array_delete(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  op_args a;
  if (!op_target(env, argv, argc, 0, &a)) return NULL;
  uint32_t index = 0, length = 0;
  if (argc < 5 || napi_get_value_uint32(env, argv[3], &index) != napi_ok ||
      napi_get_value_uint32(env, argv[4], &length) != napi_ok) {
    op_free(&a);
    napi_throw_type_error(env, NULL, "arrayDelete(doc, root, parentKey, index, length)");
    return NULL;
  }
  int rc = ycrdt_array_delete(a.d, a.root, a.pkey, index, length);
  op_free(&a);
  return rc == YCRDT_OK ? NULL : throw_rc(env, rc);
}

/* mapTypeAt(doc, root, key) → type ref of the shared type under root[key], -1 if none (YMap.get) */
static napi_value js_map_type_at(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[4], v;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 3) { napi_throw_type_error(env, NULL, "mapTypeAt(doc, root, key)"); return NULL; }
  napi_get_null(env, &argv[3]);
  napi_value args[4] = {argv[0], argv[1], argv[3], argv[2]};  /* (doc, root, null, key) */
  op_args a;
  if (!op_target(env, args, 4, 1, &a)) return NULL;
  int32_t tr = -1;
  int rc = ycrdt_map_type_at(a.d, a.root, a.key, &tr);
  op_free(&a);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  CHECK(env, napi_create_int32(env, tr, &v));
  return v;
}

/* per-key reads: JSON text, or undefined when absent / `undefined` (state 0 / 2); mapHas → bool */
static napi_value read_result(napi_env env, int rc, int state, ycrdt_out *o, int want_has) {
  napi_value v;
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  if (want_has) CHECK(env, napi_get_boolean(env, state != 0, &v));
  else if (state == 1) CHECK(env, napi_create_string_utf8(env, (const char *)o->ptr, o->len, &v));
  else CHECK(env, napi_get_undefined(env, &v));
  ycrdt_free(o);
  return v;
}

/* mapGet(doc, root, parentKey, key) → JSON text | undefined   (YMap.get, crdt.js:424) */
static napi_value js_map_get(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  op_args a;
  if (!op_target(env, argv, argc, 1, &a)) return NULL;
  int state = 0;
  ycrdt_out o = {NULL, 0};
  int rc = ycrdt_map_get(a.d, a.root, a.pkey, a.key, &state, &o);
  op_free(&a);
  return read_result(env, rc, state, &o, 0);
}

/* mapHas(doc, root, parentKey, key) → bool   (YMap.has, crdt.js:423) */
static napi_value js_map_has(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  op_args a;
  if (!op_target(env, argv, argc, 1, &a)) return NULL;
  int state = 0;
  ycrdt_out o = {NULL, 0};
  int rc = ycrdt_map_get(a.d, a.root, a.pkey, a.key, &state, &o);
  op_free(&a);
  return read_result(env, rc, state, &o, 1);
}

/* mapSize(doc, root, parentKey) → number   (YMap.size) */
static napi_value js_map_size(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3], v;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  op_args a;
  if (!op_target(env, argv, argc, 0, &a)) return NULL;
  uint32_t n = 0;
  int rc = ycrdt_map_size(a.d, a.root, a.pkey, &n);
  op_free(&a);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  CHECK(env, napi_create_uint32(env, n, &v));
  return v;
}

/* arrayLength(doc, root, parentKey) → number   (YArray.length; push, crdt.js:427) */
static napi_value js_array_length(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3], v;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  op_args a;
  if (!op_target(env, argv, argc, 0, &a)) return NULL;
  uint64_t n = 0;
  int rc = ycrdt_array_length(a.d, a.root, a.pkey, &n);
  op_free(&a);
  if (rc != YCRDT_OK) return throw_rc(env, rc);
  CHECK(env, napi_create_double(env, (double)n, &v));
  return v;
}

/* arrayGet(doc, root, parentKey, index) → JSON text | undefined   (YArray.get) */
static napi_value js_array_get(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  op_args a;
  if (!op_target(env, argv, argc, 0, &a)) return NULL;
  int64_t index = 0;
  if (argc < 4 || napi_get_value_int64(env, argv[3], &index) != napi_ok) {
    op_free(&a);
    napi_throw_type_error(env, NULL, "arrayGet(doc, root, parentKey, index)");
    return NULL;
  }
  int state = 0;
  ycrdt_out o = {NULL, 0};
  int rc = index < 0 ? YCRDT_OK : ycrdt_array_get(a.d, a.root, a.pkey, (uint64_t)index, &state, &o);
  op_free(&a);
  return read_result(env, rc, state, &o, 0);
}

static napi_value init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"setDevice", NULL, js_set_device, NULL, NULL, NULL, napi_default, NULL},
      {"docCreate", NULL, js_doc_create, NULL, NULL, NULL, napi_default, NULL},
      {"applyUpdates", NULL, js_apply_updates, NULL, NULL, NULL, napi_default, NULL},
      {"applyUpdatesMulti", NULL, js_apply_updates_multi, NULL, NULL, NULL, napi_default, NULL},
      {"encodeStateAsUpdate", NULL, js_encode_state_as_update, NULL, NULL, NULL, napi_default, NULL},
      {"encodeStateVector", NULL, js_encode_state_vector, NULL, NULL, NULL, napi_default, NULL},
      {"mergeUpdates", NULL, js_merge_updates, NULL, NULL, NULL, napi_default, NULL},
      {"diffUpdate", NULL, js_diff_update, NULL, NULL, NULL, napi_default, NULL},
      {"diffUpdates", NULL, js_diff_updates, NULL, NULL, NULL, napi_default, NULL},
      {"takeLocalUpdate", NULL, js_take_local_update, NULL, NULL, NULL, napi_default, NULL},
      {"trackLocalUpdates", NULL, js_track_local, NULL, NULL, NULL, napi_default, NULL},
      {"lastStats", NULL, js_last_stats, NULL, NULL, NULL, napi_default, NULL},
      {"version", NULL, js_version, NULL, NULL, NULL, napi_default, NULL},
      {"mapTypeAt", NULL, js_map_type_at, NULL, NULL, NULL, napi_default, NULL},
      {"docJson", NULL, js_doc_json, NULL, NULL, NULL, napi_default, NULL},
      {"typeJson", NULL, js_type_json, NULL, NULL, NULL, napi_default, NULL},
      {"mapEntries", NULL, js_map_entries, NULL, NULL, NULL, napi_default, NULL},
      {"mapSet", NULL, js_map_set, NULL, NULL, NULL, napi_default, NULL},
      {"mapSetType", NULL, js_map_set_type, NULL, NULL, NULL, napi_default, NULL},
      {"mapDelete", NULL, js_map_delete, NULL, NULL, NULL, napi_default, NULL},
      {"arrayInsert", NULL, js_array_insert, NULL, NULL, NULL, napi_default, NULL},
      {"arrayDelete", NULL, js_array_delete, NULL, NULL, NULL, napi_default, NULL},
      {"mapGet", NULL, js_map_get, NULL, NULL, NULL, napi_default, NULL},
      {"mapHas", NULL, js_map_has, NULL, NULL, NULL, napi_default, NULL},
      {"mapSize", NULL, js_map_size, NULL, NULL, NULL, napi_default, NULL},
      {"arrayLength", NULL, js_array_length, NULL, NULL, NULL, napi_default, NULL},
      {"arrayGet", NULL, js_array_get, NULL, NULL, NULL, napi_default, NULL},
  };
  napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)

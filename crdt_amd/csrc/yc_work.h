// yc_work.h — device workspace of one batched merge and the host-side launch entry points.
//
// Every array lives in HBM for the lifetime of the engine (grow-only arena, no hipMalloc on the
// merge path). Naming: B = batch bytes, G = decode groups, S = decoded structs, NC = clients,
// U = units (one per (client, clock) in the merged store), NS = segments, NO = output structs.
#pragma once
#include <initializer_list>
#include "yc_common.h"
#include "yc_view.h"

namespace yc {

struct Counters {            // device-side counters, read back at the few host sync points
  uint32_t err;              // first error code (ERR_*)
  uint32_t err_info;         // position / index that raised it
  uint32_t nsections;        // appended by the walker
  uint32_t xchunks;          // chunks of updates handed to the exit tables (xlist)
  uint32_t nds;              // decoded delete-set ranges
  uint32_t ndsclients;       // delete-set client headers
  uint32_t nstructs;         // S
  uint32_t nclients;         // NC
  uint32_t nunits_lo;        // U (low 32 bits)
  uint32_t nunits_hi;        // U (high bits; must be 0)
  uint32_t nsegs;            // NS
  uint32_t nout;             // NO
  uint32_t changed;          // pointer-jumping convergence flag
  uint32_t out_bytes;        // encoded output size (mergeUpdates / diffUpdate)
  uint32_t sv_bytes;         // encoded state-vector size
  uint32_t nkeys;            // distinct map keys
  uint32_t nruns;            // delete-set runs in the output
  uint32_t narray;           // YArray list members (segments)
  uint32_t nmapx;            // 1: a YMap entry needs full YATA (an entry item with a right origin, k_resolve)
  uint32_t any_rorigin;      // 1: a decoded item has a right origin (only then can nmapx be set)
  uint32_t ds_big;           // updates whose delete set has more ranges than one wavefront applies (DSA_WAVE), listed in ds_biglist
  uint32_t nsd_defer;        // structs k_struct_decode deferred to k_struct_decode_deferred
  uint32_t any_json;         // 1: a decoded struct holds ContentJSON / Embed / Format (k_json_structs checks them)
  uint32_t narray_roots;     // 1: a decoded item may root a YArray list (parent given, no parentSub)
  uint32_t tgroups;          // sibling groups of the YArray origin trees (yc_yata.hip)
  uint32_t tbig;             // groups too large for one lane
  uint32_t ds_region;        // Σ per-update delete-set regions (sizes the range arrays)
  uint32_t nested;           // 1: a decoded item names a parent ITEM (nested types exist)
  uint32_t nroots_sh[NSHARD]; // items with an explicit parent, sharded by workgroup (summed on the host)
  uint32_t nroots;           // items with an explicit parent (bound on the distinct lists: key table size)
  uint32_t pad[12];          // encode scratch (see yc_encode.hip)
  uint32_t climb_open[40];   // per pointer-jumping round of the YArray climb: pairs still open (yc_yata.hip)
  uint32_t sync_changed[8];  // per k_sync round: some chunk's chain exit changed (yc_decode.hip)
  uint32_t noncanon;          // lazy decode: an update's sections are not in strictly descending client order
  uint32_t lz_blocks;         // serial lazy merge: output sections
  uint32_t njson;             // JSON-like contents not in JSON.stringify's form (k_json_structs: listed in jlist)
  uint32_t ds_ntails;         // long delete-set runs whose tails k_ds_tails flags (ds_tails)
  unsigned long long out_total; // encoded output size (integrate encoder; 64-bit)
  unsigned long long ds_base;   // integrate encoder: byte position of the delete-set section
  unsigned long long items;  // Σ clock lengths of Skip structs (items = Σ all lengths − this)
  unsigned long long units;  // U = cl_base[NC] (copied on the device before a counter read)
  unsigned long long in_len; // Σ input clock lengths = s_lenscan[S] (same)
};

struct DsRange {             // one decoded (client, clock, len) delete-set range
  uint32_t client;           // value; later rewritten to cidx
  uint32_t clock;
  uint32_t len;
  uint32_t upd;
};

// Batches larger than 4 GiB are laid out in WINDOWS of 2^32 bytes: window k holds the bytes
// [k << 32, (k + 1) << 32) of the batch buffer, an update never straddles two windows, and every
// byte position a kernel handles (struct / content / section positions, chunk bounds) is a u32
// relative to its window. A kernel working on one update rebases its byte and bitmap pointers to
// the update's window once (win_bytes / win_words) and keeps the 32-bit arithmetic; a kernel that
// reaches a struct's bytes by struct index takes the window from s_win (struct_bytes).
// (The window size is 2^win_shift with win_shift = 32; tests shrink it through YCRDT_WIN_SHIFT to
// run every multi-window path on a few megabytes.)
constexpr uint32_t WIN_SHIFT = 32;
// bytes of a window updates may fill: the rest is slack for the parsers' reads past an update end
__host__ __device__ inline uint64_t win_use(uint32_t shift) {
  return (1ull << shift) - (shift >= 28 ? (1ull << 20) : (1ull << 12));
}

struct Work {
  // ---- batch input
  const uint8_t* bytes = nullptr;  // every update starts at a 64-byte aligned offset of its window
  uint64_t nbytes = 0;             // span of the batch buffer (windows before the last are 2^32 each)
  uint32_t nwin = 1;               // windows of the batch (1: every position is absolute)
  uint32_t win_shift = WIN_SHIFT;  // window size 2^win_shift
  const uint32_t* uwin = nullptr;  // [nupd] window of every update (nullptr: one window)
  const uint32_t* uoff = nullptr;  // [nupd+1] update start offsets within their windows (aligned)
  const uint32_t* ulen = nullptr;  // [nupd] real update lengths
  const uint32_t* ugroup = nullptr;// [nupd] first decode chunk of each large update
  uint32_t nupd = 0;
  const uint32_t* udoc = nullptr;  // [nupd] document of every update (multi-document batches); nullptr = one doc
  uint32_t ndocs = 1;
  const uint32_t* ulist = nullptr; // [nbig] updates on the chunk path, then [nsmall] parsed directly
  uint32_t nbig = 0, nsmall = 0;
  uint32_t small_max = 0;          // the longest of the [nsmall] updates (host-known: k_wlen's grid, k_wrank's LDS)
  uint32_t* fwsec = nullptr;       // [2 cap_sections] k_fastwalk_multi: each section's chain range [q, e)
  uint4* fwc = nullptr;            // record mode (k_fwc): per byte of a multi-section large update, the section
                                   // step from a header there {next header, chain range end, walked, why}
  const uint32_t* fwc_off = nullptr; // [nupd] record base of each record-mode update, NONE otherwise (null: none)
  uint32_t* rtab = nullptr;        // record mode: chain_len at every byte of those updates (k_rtab), indexed as fwc
  uint4* rk = nullptr;             // [nupd] record mode: the ranked last section (first struct, n, section, 1)
  uint32_t dbg_bounds = 0;         // YCRDT_DEBUG_BOUNDS=1: table indexes of the unit passes and the single-workgroup
                                   // kernels checked against their tables' sizes (bounds_fail: a message + ERR_CAPACITY)
  uint32_t fwc_walk = 256;         // k_fwc's walk bound (YCRDT_FWC_WALK; at FWM_WALK the walker never re-evaluates a chain-position header)
  uint16_t* wlen = nullptr;        // [nsmall * 16384] few small updates: the chain step at every position (k_wlen)
  uint32_t schunk = SCHUNK;        // chunk bytes of this batch's large updates (<= SCHUNK)
  uint32_t force_xtab = 0;         // YCRDT_DECODE=xtab: every large update takes the exit-table walk (tests)
  uint32_t fwm_max = 0;            // YCRDT_FWM_MAX=n: k_fastwalk_multi vouches for at most n sections per update (tests: k_walk resumes)
  uint32_t spec_hint = 2;          // k_spec chunk-start hints: 0 never, 1 always, 2 single-section updates
  uint32_t lazy = 0;               // 1: mergeUpdates / diffUpdate decode (references kept raw)
  unsigned long long* dbg = nullptr; // YCRDT_DEBUG_YATA=1: k_yata work counters
  const Group* groups = nullptr;   // [G] chunks of the large updates
  uint32_t ngroups = 0;
  // ---- capacities
  uint32_t cap_structs = 0, cap_sections = 0, cap_ds = 0, cap_dsclients = 0;
  uint64_t cap_units = 0;
  // ---- decode
  Counters* ctr = nullptr;
  uint64_t* spec_bits = nullptr;   // [B/64] positions visited by the chunk chains (large updates)
  uint32_t* cexit = nullptr;       // [G] first chain position at / past each chunk's end
  uint32_t* sexit = nullptr;       // [G] the same after k_sync's odd rounds (the even rounds write cexit)
  uint32_t* sent = nullptr;        // [2G] k_sync: the entry each chunk was last walked from; then "entered past its end" flags
  uint32_t* xtab = nullptr;        // [G x XK] locked updates only, per entry offset: count << 16 | exit - chunk end
  uint32_t* tentry = nullptr;      // [G] locked updates: true entry of a chunk the table walk did not parse
  uint32_t* xlist = nullptr;       // [G] the chunks of the locked updates (k_xtab / k_xmark work list)
  uint32_t* ccnt = nullptr;        // [G+1] chain positions per chunk (k_chunk_counts)
  uint32_t* coff = nullptr;        // [G+1] 1: the chunk's entry may be off the one chain
  uint64_t* cpre = nullptr;        // [G+1] exclusive scan of ccnt (the fast walks' chunk search)
  uint32_t* opre = nullptr;        // [G+1] exclusive scan of coff
  uint32_t* fw = nullptr;          // [2 nupd] fast-walked updates: first chain position past the exact walk, end of the last struct
  uint32_t* ufail = nullptr;       // [nupd] 1: the speculative walk gave up (locked chain phases), tables next;
                                   // 2 / 3 fast-walked, 4 / 5 resumed by k_walk, UF_PRE decoded by its marks,
                                   // UF_WALKED walked whole by k_prewalk
  uint32_t upre = 0xFFFFFFFFu;     // the update decoded by its marks (k_predecoded), NONE: none
  uint32_t walk_only = 0;          // 1: every large update is pre-decoded or pre-walked whole (no chunk walk)
  uint64_t* final_bits = nullptr;  // [B/64] verified struct starts
  uint64_t* sec_bits = nullptr;    // [B/64] first struct of every non-empty section
  uint32_t* dsstart = nullptr;     // [nupd] byte position of the delete set
  Section* sections = nullptr;     // [cap_sections] (walker order)
  uint32_t* sec_sorted = nullptr;  // [cap_sections] section index by position rank
  uint32_t* sec_uend = nullptr;    // [cap_sections] the section's update end (k_section_rank; the struct decode's bound)
  uint32_t* sec_doc = nullptr;     // [cap_sections] the section's document (multi-document batches)
  uint32_t* wcnt = nullptr;        // [B/64 + 1] popcount prefix of final_bits words
  uint32_t* wsec = nullptr;        // [B/64 + 1] popcount prefix of sec_bits words
  DsRange* ds = nullptr;           // [cap_ds] dense delete-set ranges
  DsRange* ds_tmp = nullptr;       // [cap_ds] per-update regions (decode output)
  uint32_t* ds_region = nullptr;   // [nupd+1] region offsets (scan of (ds bytes + 1) / 2)
  uint32_t* ds_count = nullptr;    // [nupd+1] ranges decoded per update
  uint32_t* ds_dense_off = nullptr;// [nupd+1] scan of ds_count
  uint32_t* ds_len = nullptr;      // [cap_ds+1] clipped lengths (scan input)
  uint32_t* jlist = nullptr;       // [jcap] structs whose JSON-like content Yjs would write back differently (k_json_structs)
  uint32_t jcap = 0;
  uint32_t ntrusted = 0;           // the first ntrusted staged updates are doc states the engine wrote: never rewritten
  uint32_t jskip_any = 0;          // 1: a rewrite pass ran: `any` contents are not rewritten again (readAny o writeAny
                                   //    is not idempotent: an own "__proto__" member written by writeAny)
  uint4* ds_tails = nullptr;       // [DS_TAILS_CAP] (first unit lo, hi, units) of long delete-set runs past their first
                                   // DS_TAIL_MIN units: flagged grid-wide by k_ds_tails (set only with a large delete set)
  uint32_t* ds_biglist = nullptr;  // [nupd] updates with more than DSA_WAVE ranges (ctr->ds_big of them): k_units spreads
                                   // their ranges past the first DSA_WAVE over extra workgroups, whichever decoder read them
  // large delete sets decoded grid-wide (yc_decode.hip k_dsp_*): per chunk of the large updates
  // the terminal bytes (varuint ends) of its delete-set part and their scan; every varuint's value;
  // the client blocks (value index of the client, client, ranges, first range) of each update
  uint32_t* dsp_cnt = nullptr;     // [G+1] terminal bytes of the chunk's delete-set part
  uint32_t* dsp_pre = nullptr;     // [G+1] exclusive scan of dsp_cnt
  uint32_t* dsp_val = nullptr;     // [2 cap_ds] varuint values, update u's at 2 ds_region[u]
  uint4* dsp_blk = nullptr;        // [nbig x DSP_MAXBLK] client blocks of big update b
  uint32_t* dsp_b = nullptr;       // [nupd] big index of an update whose delete set took the grid path, NONE: the wavefront's
  uint32_t* dsp_nb = nullptr;      // [nbig] its client blocks
  uint32_t* dsp_gb = nullptr;      // [nbig+1] scan of the delete-set chunks of each big update (the grid's work list)
  uint32_t* dsp_fail = nullptr;    // [nupd] a varuint longer than 6 bytes: the wavefront decodes (and reports) it
  uint32_t* dsp_j = nullptr;       // [2 cap_ds] per delete-set value index: where 32 header hops from it land (k_dsh_jump)
  uint32_t* dsp_js = nullptr;      // [2 cap_ds] the run counts those hops pass
  uint2* dsp_h = nullptr;          // [nbig x (DSH_SEG + 1)] every 32nd header (value index, runs before it); [DSH_SEG]: (failed, runs)
  uint32_t dsh_grid = 0;           // k_dsh_jump's workgroups per big update
  uint64_t* ds_scan = nullptr;     // [cap_ds+1]
  uint32_t* dsclient_vals = nullptr; // [cap_dsclients] (client values seen in delete sets)
  // ---- per struct (S)
  uint32_t* s_pos = nullptr;       // first byte (within the struct's window)
  uint8_t* s_win = nullptr;        // window of the struct's bytes (written only when nwin > 1)
  uint32_t* s_sec = nullptr;       // index into sections
  uint32_t* s_len = nullptr;
  uint64_t* s_lenscan = nullptr;   // [S+1] exclusive prefix of s_len
  uint32_t* s_clock = nullptr;
  uint32_t* s_cidx = nullptr;
  uint8_t* s_info = nullptr;
  uint32_t* s_ocidx = nullptr;     // origin client index (NONE = no origin)
  uint32_t* s_oclock = nullptr;
  uint32_t* s_rcidx = nullptr;     // right origin client index
  uint32_t* s_rclock = nullptr;
  uint8_t* s_pk = nullptr;         // parent kind: 0 inherited, 1 root type name, 2 parent item id
  uint32_t* s_pa = nullptr;        // pk 1: name varString position; pk 2: parent client index
  uint32_t* s_pb = nullptr;        // pk 1: name varString length;   pk 2: parent clock
  uint32_t* s_psub = nullptr;      // parentSub varString position or NONE
  uint32_t* s_psublen = nullptr;
  uint32_t* s_cpos = nullptr;      // content byte range
  uint32_t* s_cend = nullptr;
  uint32_t* s_celem = nullptr;     // position of first Any/JSON element (after the count varuint)
  uint32_t* sd_defer = nullptr;    // [S] structs whose decode k_struct_decode deferred (nested `any`, ContentDoc)
  // ---- clients (NC)
  uint32_t* cl_vals = nullptr;     // sorted distinct client ids [cap_sections]
  uint64_t* cl_key = nullptr;      // multi-doc: sorted distinct (doc << 32 | client) keys; cl_vals = their low words
  uint64_t* cl_key2 = nullptr;     // multi-doc sort scratch
  uint64_t* ch_key = nullptr;      // client hash: (doc << 32 | client) per slot, ~0 = empty (null until built)
  uint32_t* ch_val = nullptr;      // client hash: client index per slot
  uint32_t ch_mask = 0;            // slots - 1 (a power of two >= 2 x the clients)
  uint32_t* cl_doc = nullptr;      // document of every client index (multi-doc)
  uint32_t* cl_tmp = nullptr;      // sort scratch [cap_sections]
  uint32_t* cl_state = nullptr;
  uint8_t* cl_single = nullptr;    // [NC] 1: the client's structs come from one section of one update    // per client state (max end clock)
  uint64_t* cl_base = nullptr;     // [NC+1] exclusive prefix of states (unit base)
  uint32_t* cl_start = nullptr;    // per client start clock for diff encodes (sv); 0 = full
  uint32_t delta = 0;              // 1: some cl_start is nonzero (a delta encode against a state vector)
  // per-client integration caps (Yjs pending structs, yc_ingest.h): sorted (client, cap) pairs;
  // units at or past a client's cap are left out of the merge and delete-set ranges clipped to it
  const uint32_t* cap_client = nullptr;
  const uint32_t* cap_clock = nullptr;
  uint32_t ncaps = 0;
  uint32_t capped = 0;             // 1: caps given (clip silently); 0: anything missing is ERR_PENDING
  // ---- per unit (U)
  uint32_t* u_owner = nullptr;
  uint32_t* u_flags = nullptr;
  uint64_t* u_cutbits = nullptr;   // [U/64+1]
  uint32_t* u_wpre = nullptr;      // [U/64+2] popcount prefix of u_cutbits words
  // ---- per segment (NS <= U)
  uint32_t* g_start = nullptr;     // first unit (global unit index)
  uint32_t* g_cidx = nullptr;
  uint32_t* g_src = nullptr;       // owning struct
  uint32_t* g_flags = nullptr;     // SEG_* flags
  uint32_t* g_origin = nullptr;    // origin unit (global) or NONE
  uint32_t* g_rorigin = nullptr;   // right-origin unit or NONE
  uint4* g_hop = nullptr;          // key resolution record {flags, climbing key, link, origin segment}:
                                   // one 16-B line per climbing hop (k_seg_props -> k_resolve)
  uint32_t* g_key = nullptr;       // resolved key slot or NONE
  uint32_t* g_maxchild = nullptr;  // seg + 1 of the max-client child (segments are in client order), 0 = none
  uint32_t* g_next = nullptr;      // descent pointer / pointer jumping
  uint32_t* g_outid = nullptr;     // output struct id (scan of !merge flags)
  uint32_t* g_tmp = nullptr;       // scratch per segment
  uint32_t* g_tmp2 = nullptr;
  // ---- keys (hash table)
  uint64_t* k_hash = nullptr;      // [cap_keys] open addressing table: (claiming root struct + 1) << 32 | low
                                   // half of the list hash (0 = empty); lists compared by name (key_insert)
  uint64_t key_mask = ~0ull;       // list-hash bits kept (YCRDT_KEY_HASH_BITS: tests force collisions)
  uint32_t* k_rootmax = nullptr;   // [cap_keys] seg + 1 of the max-client root, 0 = none
  uint32_t* k_winner = nullptr;    // [cap_keys] winning (rightmost) segment
  uint32_t* k_parent = nullptr;    // [cap_keys] parent type item unit (NONE = root type)
  uint32_t* k_flags = nullptr;     // [cap_keys] KF_* flags
  uint32_t cap_keys = 0;
  // ---- YArray lists (YATA integration, yc_yata.hip)
  uint32_t* g_right = nullptr;     // [NS] right neighbour after integration (NONE = end of list)
  uint32_t* y_key = nullptr;       // [NS] sort key: key slot of live array-list segments, NONE otherwise
  uint32_t* y_keys = nullptr;      // [NS] sorted keys
  uint32_t* y_seg = nullptr;       // [NS] segments sorted by (key slot, segment)
  uint32_t* y_iota = nullptr;      // [NS] 0..NS-1 (sort values)
  uint32_t* y_lstart = nullptr;    // [lists+1] first position of every list in y_seg
  uint32_t* y_state = nullptr;     // [NS] integration state / stamps (per segment)
  uint32_t* y_before = nullptr;    // [NS]
  uint32_t* y_confl = nullptr;     // [NS]
  uint32_t* y_stack = nullptr;     // [NS]
  // ---- parallel YATA as an origin-tree pre-order (yc_yata.hip)
  uint32_t* t_key = nullptr;       // [NS] sibling-group key: origin segment, or NS + list slot for roots; NONE = not in a list
  uint32_t* t_keys = nullptr;      // [NS] sorted keys
  uint32_t* t_seg = nullptr;       // [NS] segments sorted by (group, segment): siblings in client order
  uint32_t* t_pos = nullptr;       // [NS] segment -> sorted position
  uint32_t* t_gstart = nullptr;    // [groups+1] first sorted position of every sibling group
  uint32_t* t_next = nullptr;      // [NS] next sibling (sorted position) after the sibling loops
  uint32_t* t_done = nullptr;      // [NS] sibling-loop state (0 pending, 1 on the stack, 2 placed)
  uint32_t* t_first = nullptr;     // [NS] first child segment of every segment (NONE = leaf)
  uint32_t* t_nsib = nullptr;      // [NS] next sibling segment (NONE = last child)
  uint32_t* t_jump = nullptr;      // [NS] climbing link: an ancestor with the same "next in pre-order"
  uint32_t* t_big = nullptr;       // [groups] ids of the groups too large for one lane
  uint32_t* t_prv = nullptr;       // [NS] previous sibling (sorted position) during the loops
  uint32_t* t_mprv = nullptr;      // [NS] previous member of the same right-origin group
  uint32_t* t_mtail = nullptr;     // [NS] last member of the group whose right origin is this sibling
  uint32_t* t_otail = nullptr;     // [NS] last member of the outside-right-origin group anchored here
  uint32_t* t_hkey = nullptr;      // [2 NS + 4] huge sibling groups: anchor hash keys (right-origin units)
  uint32_t* t_hval = nullptr;      // [2 NS + 4]   its first member (lowest group position)
  uint32_t* t_flag = nullptr;      // [NS + 2]   chain starts of a huge group, then their scan
  uint32_t* t_trep = nullptr;      // [NS] anchor of the member's right-origin group
  // ---- lazy merge (mergeUpdates / diffUpdate, yc_lazy.hip)
  uint32_t* usec_start = nullptr;  // [nupd] first section of every update (walker order)
  uint32_t* usec_n = nullptr;      // [nupd] sections of every update
  uint64_t* lz_key = nullptr;      // [sections] (client rank, update)
  uint64_t* lz_keys = nullptr;     // sorted
  uint32_t* lz_iota = nullptr;
  uint32_t* lz_sec = nullptr;      // sections sorted by (client desc, update)
  uint32_t* lz_rstart = nullptr;   // [NC+1] readers of every client rank
  uint32_t* lz_prev = nullptr;     // [sections] previous non-empty section of the same update
  uint32_t* lz_first = nullptr;    // [sections] first non-Skip struct
  uint32_t* lz_cap = nullptr;      // [blocks+1] event slots per output block
  uint32_t* lz_evbase = nullptr;   // [blocks+1] exclusive scan of lz_cap
  uint32_t* lz_evn = nullptr;      // [blocks] events emitted
  uint32_t* lz_flag = nullptr;     // [sections] leave stamp published
  uint32_t* lz_leave_hi = nullptr; // [sections] leave stamp (client rank + 1, step)
  uint32_t* lz_leave_lo = nullptr;
  uint32_t lz_nblk = 0, lz_diff = 0;
  uint32_t lz_multi = 0;            // 1: one diffUpdate per input update (sync responder batch); no global headers
  uint32_t* lz_bclient = nullptr;   // serial lazy merge: client of every output section (null: per-client blocks)
  uint32_t* ev_kind = nullptr;     // [slots] REF_GC | REF_SKIP | 1 (item)
  uint32_t* ev_src = nullptr;
  uint32_t* ev_clock = nullptr;
  uint32_t* ev_len = nullptr;
  uint32_t* ev_size = nullptr;     // [slots+1]
  uint32_t* ev_pos = nullptr;      // [slots+1]
  uint32_t* blk_size = nullptr;    // [blocks+1]
  uint32_t* blk_pos = nullptr;     // [blocks+1]
  const uint32_t* sv_client = nullptr;  // diff target state vector, sorted by client
  const uint32_t* sv_clock = nullptr;
  uint32_t sv_n = 0;
  const uint32_t* sv_off = nullptr; // lz_multi: [nupd+1] each update's range of (sv_client, sv_clock)
  uint64_t* dsm_key = nullptr;     // [ds] (~client, clock)
  uint64_t* dsm_keys = nullptr;
  uint32_t* dsm_len = nullptr;
  uint32_t* dsm_lens = nullptr;
  uint64_t* dsm_end = nullptr;     // (~client, clock + len)
  uint64_t* dsm_max = nullptr;     // segmented running max
  uint32_t* dsm_flag = nullptr;    // [ds+1]
  uint32_t* dsm_rid = nullptr;     // [ds+1]
  uint32_t* dr_client = nullptr;   // [runs] delete-set runs in output order
  uint32_t* dr_clock = nullptr;
  uint32_t* dr_end = nullptr;
  uint32_t* dw_flag = nullptr;     // [runs+1]
  uint32_t* dw_gid = nullptr;      // [runs+1]
  uint32_t* dw_gstart = nullptr;   // [runs+1]
  uint32_t* dw_size = nullptr;     // [runs+1]
  uint32_t* dw_pos = nullptr;      // [runs+1]
  // Yjs 13.5.16 (compat 135) writes a delete set's clients in Map insertion order: first appearance
  // (readDeleteSet / mergeDeleteSets, per update for a multi diff). ds_fa[i] = index of the first
  // range of range i's client; keys then carry ds_fa instead of ~client.
  uint32_t ds_first = 0;
  uint32_t* ds_fa = nullptr;       // [ds]
  // ---- encode (NO <= NS)
  uint32_t* o_first = nullptr;     // [NO+1] first segment of output struct (+ sentinel)
  uint32_t* o_cidx = nullptr;      // client of output struct
  uint32_t* o_size = nullptr;      // encoded size (0 = below the target state vector)
  uint32_t* o_pos = nullptr;       // [NO+1] exclusive prefix of o_size
  uint8_t* o_gen = nullptr;        // [NO] 1: the general encoder takes the output struct (k_out_sizes_general)
  uint32_t* r_seg = nullptr;       // [runs] first segment of delete-set run
  uint32_t* r_len = nullptr;       // [runs] run length in units
  uint32_t* r_size = nullptr;      // [runs+1] encoded size of (clock,len)
  uint32_t* r_pos = nullptr;       // [runs+1]
  uint32_t* cc = nullptr;          // per-client scratch: CC_N arrays of (cap_clients+1)
  uint64_t* cc64 = nullptr;        // per-client byte positions (64-bit): CC64_N arrays of (cap_clients+1)
  // compat 135: delete-set / state-vector client order = the doc store's insertion order.
  // cl_emit[slot] = client table index written at that slot, cl_slot = its inverse (null: desc)
  const uint32_t* cl_emit = nullptr;
  const uint32_t* cl_slot = nullptr;
  uint32_t cap_clients = 0;
  uint8_t* out = nullptr;          // encoded update
  uint64_t cap_out = 0;
  uint64_t cap_sv = 0;
  uint8_t* sv_out = nullptr;       // encoded state vector
  uint32_t* scratch = nullptr;     // scan staging (max of all scan lengths)
  // ---- rocPRIM scratch
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
};

// client index of (document, client id); NONE if the batch has no such client. Multi-document
// batches index clients by (doc, client), so every per-client structure stays per document.
// XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md,
// speed only, never correctness), so block b and b + 8 share an L2. The logical block below gives
// XCD x one contiguous 1/8 of the grid: the random gathers of a per-segment / per-struct pass
// (origins, clients, winner slots) mostly land in the same document's tables, which then stay in
// that XCD's L2 instead of being pulled into all eight. A bijection on [0, gridDim.x).
__device__ __forceinline__ uint32_t xcd_block() {
  const uint32_t b = blockIdx.x, G = gridDim.x, per = G >> 3, rem = G & 7u, x = b & 7u;
  return x * per + min(x, rem) + (b >> 3);
}
__device__ __forceinline__ uint32_t gidx() { return xcd_block() * blockDim.x + threadIdx.x; }

// Workgroups that wait on other workgroups of the same launch (decoupled look-back, the lazy
// merge's stamps) take their index in START order: ordered_block_id hands out base, base + 1, ...
// as the workgroups begin, so every index a workgroup waits on belongs to one that is already
// running. Block ids give no such guarantee: each XCD dispatches its share independently, and a
// concurrent kernel (another stream or process) filling one XCD can leave a lower block id
// undispatched behind workgroups spinning on it. Counter and base per stream (yc_prims.hip).
struct OrderedIds {
  unsigned long long* ctr = nullptr;
  unsigned long long base = 0;
};
bool ordered_ids(uint64_t nblocks, hipStream_t s, OrderedIds& out);  // one per launch, in launch order
__device__ __forceinline__ uint32_t ordered_block_id(unsigned long long* ctr, unsigned long long base) {
  __shared__ uint32_t id;
  if (threadIdx.x == 0) id = (uint32_t)(atomicAdd(ctr, 1ull) - base);
  __syncthreads();
  return id;
}

// Decoupled look-back (yc_prims.hip k_scan_lb; also inside producer kernels, whose scan then needs
// no pass of its own). A tile's state on a chain is ONE 64-bit word — epoch (22 bits) | status (2:
// aggregate / inclusive prefix) | value (40 bits) — stored and loaded as a relaxed agent-scope
// atomic (coherent across the XCDs' L2s without the invalidations an acquire costs on gfx950).
// Every launch takes a new epoch, so states left by earlier launches read as "not yet".
constexpr uint64_t LB_VAL = (1ull << 40) - 1;
struct LbChains {                       // one launch's look-back chains (lb_launch, yc_prims.hip)
  unsigned long long* state = nullptr;  // chain c's tile states at state + c * stride
  uint64_t stride = 0;
  uint32_t epoch = 0;
  unsigned long long* ord = nullptr;    // ordered tile ids (ordered_block_id)
  unsigned long long ord_base = 0;
};
bool lb_launch(uint64_t tiles, uint32_t chains, hipStream_t s, LbChains& out);
// One full wavefront: publishes `tile`'s aggregate, looks back 64 tiles per round (each lane
// spinning on its own predecessor) to the nearest inclusive prefix, publishes its own inclusive
// prefix, and returns the tile-exclusive prefix (mod 2^40) in every lane. Tiles wait only on
// lower ordered ids, which are running.
__device__ __forceinline__ uint64_t lb_wave_lookback(unsigned long long* __restrict__ state, uint32_t tile, uint32_t epoch, uint64_t agg) {
  const uint32_t lane = threadIdx.x & 63;
  const unsigned long long ep = (unsigned long long)epoch << 42;
  if (tile == 0) {
    if (lane == 0) __hip_atomic_store(&state[0], ep | (2ull << 40) | (agg & LB_VAL), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0) __hip_atomic_store(&state[tile], ep | (1ull << 40) | (agg & LB_VAL), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t pre = 0;
  for (int64_t j = (int64_t)tile - 1;; j -= 64) {
    const int64_t me = j - (int64_t)lane;
    uint32_t st = 2;
    uint64_t val = 0;
    if (me >= 0) {
      unsigned long long x;
      while (((x = __hip_atomic_load(&state[me], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 42) != epoch)
        __builtin_amdgcn_s_sleep(1);
      st = (uint32_t)(x >> 40) & 3u;
      val = x & LB_VAL;
    }
    const uint64_t done = __ballot(st == 2);  // lanes past tile 0 count as done with 0
    const uint32_t stop = (uint32_t)__ffsll((long long)done) - 1;  // nearest inclusive prefix
    uint64_t part = lane <= stop ? val : 0ull;
    for (uint32_t off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
    pre += part;
    if (done) break;
  }
  if (lane == 0) __hip_atomic_store(&state[tile], ep | (2ull << 40) | ((pre + agg) & LB_VAL), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return pre;
}

__device__ __forceinline__ uint64_t client_hash(uint64_t k) {  // splitmix64 finaliser
  k ^= k >> 30; k *= 0xBF58476D1CE4E5B9ull;
  k ^= k >> 27; k *= 0x94D049BB133111EBull;
  return k ^ (k >> 31);
}
// client index of (doc, client) or NONE: one or two probes of the client hash once it is built
// (decode builds it right after the client table), a binary search over the sorted table before
__device__ __forceinline__ uint32_t find_client(const Work& w, uint32_t nclients, uint32_t doc, uint32_t client) {
  if (w.ch_key) {
    const uint64_t key = w.udoc ? (((uint64_t)doc << 32) | client) : (uint64_t)client;
    for (uint32_t slot = (uint32_t)client_hash(key) & w.ch_mask;; slot = (slot + 1) & w.ch_mask) {
      const uint64_t k = w.ch_key[slot];
      if (k == key) return w.ch_val[slot];
      if (k == ~0ull) return NONE;
    }
  }
  if (!w.udoc) {
    const uint32_t i = lower_bound_u32(w.cl_vals, nclients, client);
    return (i < nclients && w.cl_vals[i] == client) ? i : NONE;
  }
  const uint64_t key = ((uint64_t)doc << 32) | client;
  uint32_t lo = 0, hi = nclients;
  while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (w.cl_key[m] < key) lo = m + 1; else hi = m; }
  return (lo < nclients && w.cl_key[lo] == key) ? lo : NONE;
}
__device__ __forceinline__ uint32_t doc_of_update(const Work& w, uint32_t upd) { return w.udoc ? w.udoc[upd] : 0u; }
// first unit of segment s (s = NS: the sentinel U) and the segment of unit g
__device__ __forceinline__ uint32_t seg_start(const Work& w, uint32_t s) { return w.g_start[s]; }
__device__ __forceinline__ uint32_t seg_of_unit(const Work& w, uint32_t g) {
  return w.u_wpre[g >> 6] + (uint32_t)__popcll(w.u_cutbits[g >> 6] & ((2ull << (g & 63)) - 1)) - 1;
}
// ---- windows (see WIN_SHIFT): the byte and bitmap bases of window k
__device__ __forceinline__ uint32_t upd_win(const Work& w, uint32_t upd) { return w.uwin ? w.uwin[upd] : 0u; }
__device__ __forceinline__ const uint8_t* win_bytes(const Work& w, uint32_t win) { return w.bytes + ((uint64_t)win << w.win_shift); }
#define win_words(bits, win) ((bits) + ((uint64_t)(win) << (w.win_shift - 6)))  // (w: the kernel's Work)
// the bytes of struct s's window (one window: no load)
__device__ __forceinline__ const uint8_t* struct_bytes(const Work& w, uint32_t s) {
  return w.nwin > 1 ? win_bytes(w, w.s_win[s]) : w.bytes;
}

// Byte range of content elements [e0, e1) of struct `src` (ContentAny: lib0 `any` values,
// ContentJSON: varStrings, ContentString: UTF-16 code units of the UTF-8 text; every other
// content has length 1 and is copied whole). This is ContentX.splice (Y@70000..) as a byte slice.
// The element walk is out of line: inlined, the nested-`any` skipper multiplies the register
// demand (and so cuts the occupancy) of every kernel that encodes structs, for a path that only
// split structs take. The whole-content case stays inline.
// (Plain values in, the range packed in a register pair out: a reference to Work or an
// out-parameter would make every caller spill them to scratch memory on every path.)
static __device__ __attribute__((noinline)) uint64_t content_slice_walk(const uint8_t* __restrict__ by, uint32_t ref, uint32_t celem,
                                                                        uint32_t cpos, uint32_t end, uint32_t e0, uint32_t e1);
__device__ __forceinline__ bool content_slice(const Work& w, uint32_t src, uint32_t e0, uint32_t e1, uint32_t& b0, uint32_t& b1) {
  const uint32_t ref = w.s_info[src] & 31u;
  if (e0 == 0 && e1 == w.s_len[src] && (ref == REF_ANY || ref == REF_JSON)) {  // the whole content
    b0 = w.s_celem[src];
    b1 = w.s_cend[src];
    return true;
  }
  const uint64_t r = content_slice_walk(struct_bytes(w, src), ref, w.s_celem[src], w.s_cpos[src], w.s_cend[src], e0, e1);
  if (r == ~0ull) return false;
  b0 = (uint32_t)r;
  b1 = (uint32_t)(r >> 32);
  return true;
}
static __device__ __attribute__((noinline)) uint64_t content_slice_walk(const uint8_t* __restrict__ by, uint32_t ref, uint32_t celem,
                                                                        uint32_t cpos, uint32_t end, uint32_t e0, uint32_t e1) {
  uint32_t b0 = 0, b1 = 0;
  const bool got = [&]() -> bool {
  if (ref == REF_ANY || ref == REF_JSON) {
    uint32_t p = celem;
    bool ok = true;
    for (uint32_t i = 0; i < e1; ++i) {
      if (i == e0) b0 = p;
      if (ref == REF_ANY) {
        uint32_t steps = 0xFFFFFFFFu;
        ok = skip_any<32>(by, p, end, steps);
      } else {
        const uint32_t k = rd_vu(by, p, end, ok);
        if (ok) skip_bytes(p, k, end, ok);
      }
      if (!ok) return false;
    }
    if (e0 == e1) b0 = p;
    b1 = p;
    return true;
  }
  if (ref == REF_STRING) {
    uint32_t p = cpos;
    bool ok = true;
    rd_vu(by, p, end, ok);  // byte length prefix
    if (!ok) return false;
    uint32_t u = 0;  // UTF-16 units before p
    b0 = e0 == 0 ? p : NONE;
    while (p < end && u < e1) {
      const uint32_t c = by[p];
      const uint32_t n = c < 0x80u ? 1u : c < 0xE0u ? 2u : c < 0xF0u ? 3u : 4u;
      const uint32_t du = n == 4 ? 2u : 1u;
      if (u < e0 && u + du > e0) return false;  // a slice through a surrogate pair
      if (u < e1 && u + du > e1) return false;
      p += n;
      u += du;
      if (u == e0) b0 = p;
    }
    b1 = p;
    return b0 != NONE && u == e1;
  }
  b0 = cpos;
  b1 = end;
  return true;
  }();
  return got ? ((uint64_t)b1 << 32) | b0 : ~0ull;
}

// writeAny (L0@1937) of the `any` values [e0, e1) of a struct whose content is flagged
// ANY_REENCODE (yc_parse.h): containers, keys and strings with shortest-form lengths, numbers in the
// form writeAny picks for the JS number they decode to. Returns the bytes; writes them when WRITE.
// Out of line (rare): a Work reference is never taken (the callers pass plain values).
template <bool WRITE>
__device__ __attribute__((noinline)) uint32_t any_canon(const uint8_t* __restrict__ by, uint32_t p, uint32_t end, uint32_t e0,
                                                        uint32_t e1, uint8_t* __restrict__ out, uint64_t q0) {
  uint64_t q = q0;
  auto put = [&](uint32_t x) { if (WRITE) out[q] = (uint8_t)x; ++q; };
  auto put_vu = [&](uint32_t v) { while (v > 0x7Fu) { put(0x80u | (v & 0x7Fu)); v >>= 7; } put(v); };
  auto put_vi = [&](bool neg, uint32_t m) {
    put((m > 63u ? 0x80u : 0u) | (neg ? 0x40u : 0u) | (m & 63u));
    m >>= 6;
    while (m) { put((m > 127u ? 0x80u : 0u) | (m & 127u)); m >>= 7; }
  };
  auto put_num = [&](double x) {
    const uint32_t k = num_form(x);
    if (k == 0) { put(125); put_vi(x < 0 || (x == 0 && signbit(x)), (uint32_t)fabs(x)); return; }
    if (k == 1) { union { float f; uint32_t u; } c; c.f = (float)x; put(124); for (int s = 24; s >= 0; s -= 8) put((c.u >> s) & 0xFFu); return; }
    union { double d; uint64_t u; } c; c.d = x;  // (a NaN: the bits it has, as V8 writes them)
    put(123);
    for (int s = 56; s >= 0; s -= 8) put((uint32_t)(c.u >> s) & 0xFFu);
  };
  bool ok = true;
  // members left per open container level (the elements of the content are one implicit level)
  uint32_t rem[33];
  uint32_t objm = 0;  // bit d: level d is an object
  int d = 0;
  rem[0] = e1;
  uint32_t idx = 0;  // content element index at level 0
  for (;;) {
    // one value at p
    if (d == 0 && idx >= e1) break;
    const bool emit = idx >= e0;  // (constant while inside one content element)
    const uint32_t tag = by[p++];
    const uint32_t s0 = p;
    switch (tag) {
      case 127: case 126: case 121: case 120: if (emit) put(tag); break;
      case 125: {
        skip_vi(by, p, end, ok);
        bool neg;
        const uint32_t m = vi_decode(by, s0, p, neg);
        if (emit) { if (!neg && m > 0x7FFFFFFFu) put_num((double)m); else { put(125); put_vi(neg, m); } }
        break;
      }
      case 124: p += 4; if (emit) put_num(f32_of(be32(by, s0))); break;
      case 123: p += 8; if (emit) put_num(f64_of(be64(by, s0))); break;
      case 122: p += 8; if (emit) { put(122); for (uint32_t i = s0; i < p; ++i) put(by[i]); } break;
      case 119: case 116: {
        const uint32_t n = rd_vu(by, p, end, ok);
        if (emit) { put(tag); put_vu(n); for (uint32_t i = 0; i < n; ++i) put(by[p + i]); }
        p += n;
        break;
      }
      default: {  // 117 array / 118 object
        const uint32_t n = rd_vu(by, p, end, ok);
        if (emit) { put(tag); put_vu(n); }
        if (n > 0) {
          if (d >= 32) return 0;  // (the decoder's stack bound: never reached for flagged content)
          ++d;
          rem[d] = n;
          if (tag == 118) objm |= 1u << d; else objm &= ~(1u << d);
          if (tag == 118) { const uint32_t k = rd_vu(by, p, end, ok); if (emit) { put_vu(k); for (uint32_t i = 0; i < k; ++i) put(by[p + i]); } p += k; }
          continue;
        }
        break;
      }
    }
    // a value completed: pop finished levels, read the next key of an object
    for (;;) {
      if (d == 0) { ++idx; break; }
      if (--rem[d] == 0) { --d; continue; }
      if ((objm >> d) & 1u) {
        const uint32_t k = rd_vu(by, p, end, ok);
        if (idx >= e0) { put_vu(k); for (uint32_t i = 0; i < k; ++i) put(by[p + i]); }
        p += k;
      }
      break;
    }
  }
  return (uint32_t)(q - q0);
}

// YCRDT_DEBUG_BOUNDS: an index past its table (never on a correct merge: the bound every small pass
// and every unit pass sizes from) stops the merge with a capacity error instead of writing past the
// table; err_info names the check (BOUNDS_* below), the host reports it (yc_engine.hip check()).
// Inline and without printf: a call in a kernel (even one never taken) makes it keep registers
// across the call — k_units 38 -> 60 VGPRs — and a Work reference passed out of line copies the
// whole Work to scratch in every lane (k_units / k_seg_props 20 x slower; tests/test_kernel_resources.py)
enum : uint32_t { BOUNDS_UNIT = 1, BOUNDS_KEY, BOUNDS_MERGE_SMALL, BOUNDS_ENCODE_SMALL, BOUNDS_OUTPUT, BOUNDS_DECODE_TAIL, BOUNDS_SECTIONS };
__device__ __forceinline__ void bounds_fail(Counters* ctr, uint32_t what) {
  raise_err(&ctr->err, ERR_CAPACITY);
  ctr->err_info = 0xB0DE0000u | what;
}
#define YC_BOUND(w, idx, cap, what) \
  do { if ((w).dbg_bounds && (uint64_t)(idx) >= (uint64_t)(cap)) bounds_fail((w).ctr, (what)); } while (0)

// per-client scratch arrays inside Work::cc
enum : uint32_t {
  CC_FIRST_OUT = 0, CC_FIRST_INCL, CC_NINCL, CC_HDR, CC_BLK, CC_BLKPOS, CC_NRUNS, CC_FIRST_RUN,
  CC_DSBLK, CC_DSPOS, CC_SV, CC_SVPOS, CC_REV, CC_REVSCAN, CC_RUN_LO, CC_REV2, CC_REVSCAN2, CC_REV3, CC_REVSCAN3, CC_N
};

// 64-bit per-client columns inside Work::cc64: the block positions of the struct, delete-set and
// state-vector sections, and the scans they come from
enum : uint32_t { CC64_BLKPOS = 0, CC64_DSPOS, CC64_SVPOS, CC64_SCAN, CC64_SCAN2, CC64_SCAN3, CC64_N };

// segment flags
enum : uint32_t {
  SEG_DEL = 1u,        // deleted in the final state
  SEG_GC = 2u,
  SEG_EXPLICIT = 4u,   // segment starts at its source struct's first unit
  SEG_ROOT = 8u,       // explicit parent (root name) + parentSub
  SEG_MERGE = 16u,     // merges into the previous segment
  SEG_ITEM = 32u,
  SEG_ARRAY = 64u,     // member of a YArray list (no parentSub)
  SEG_PSUB = 128u,     // member of a YMap entry list (parentSub)
  SEG_OLOW = 256u,     // its client index is below its origin's (a YATA sibling placed before the
                       // origin's own-client successor: that successor cannot merge, k_seg_props)
  SEG_WIN = 512u,      // the value of its YMap entry (k_winner_walk); every other entry item is deleted
  SEG_YMAPX = 1024u,   // a YMap entry ordered by full YATA (its key has an entry item with a right
                       // origin: the max-client descent does not apply): adjacency from g_right
  SEG_HASRO = 2048u,   // (hop record only, k_seg_props -> k_resolve) the item has a right origin
};
// bit 31 of the climbing keys (g_tmp) between k_seg_props and k_resolve: the list is a YMap entry
// (key slots < 2^31); g_key holds the final slots without it
constexpr uint32_t KEY_PSUB = 0x80000000u;
// key flags
enum : uint32_t {
  KF_PSUB = 1u,        // the list is a YMap entry (items carry a parentSub)
  KF_DEAD = 2u,        // the parent type item is deleted: every member becomes GC
  KF_YATA = 4u,        // a YMap entry with an item carrying a right origin: ordered by full YATA
};
// unit flags
enum : uint32_t {
  UF_DEL = 1u,         // source content is ContentDeleted
  UF_GC = 2u,          // a GC struct covers the unit
  UF_DS = 0x100u,      // a delete-set range covers the unit (byte 1: set by a plain byte store)
  UF_CUT = 0x10000u,   // a struct boundary is required before this unit (byte 2: plain byte store)
  UF_LOWCHILD = 0x1000000u,  // some YMap child of this unit has a lower client than the unit: no merge
                             // with its own-client successor (byte 3: plain byte store, k_seg_props)
};

// ---- materialised view (yc_view.hip), copied to the host as is
struct ViewBufs {
  uint32_t* kmap = nullptr;  // [cap_keys] slot -> ViewKey index
  uint32_t* krep = nullptr;  // [cap_keys] a root member segment
  ViewKey* keys = nullptr;   // [cap_keys]
  uint32_t* nkeys = nullptr;
  uint32_t* pos_of = nullptr;// [NS] segment -> sorted member position
  uint32_t *d0 = nullptr, *n0 = nullptr, *d1 = nullptr, *n1 = nullptr;  // [narr] list ranking
  uint32_t* order = nullptr; // [narr] members in document order
  ViewSeg* segs = nullptr;   // [narr]
};
void launch_view(const Work& w, const ViewBufs& v, uint32_t nsegs, uint32_t nlists, uint32_t narr, hipStream_t s);

// ---- a doc state's decode, written by the encode that produced it (k_state_marks): the next merge
// of the doc takes its state's struct / section starts, section records and delete-set start from
// here instead of parsing the state again (k_predecoded). Positions are the state's own.
constexpr uint32_t UF_PRE = 6;   // ufail of the update k_predecoded decoded
constexpr uint32_t UF_WALKED = 7;  // ufail of a large update k_prewalk decoded whole (a short struct section)
struct PreMarks {
  uint64_t* fbits = nullptr;   // [nw] struct starts
  uint64_t* sbits = nullptr;   // [nw] first struct of every non-empty section
  Section* secs = nullptr;     // [cap_secs] section record of every client slot (n = 0: no block; upd 0)
  uint32_t* meta = nullptr;    // [3] sections (non-empty blocks), delete-set start, client slots
  uint32_t nw = 0, cap_secs = 0;
};
void launch_state_marks(const Work& w, uint32_t nout, uint32_t nclients, const PreMarks& m, hipStream_t s);
// update u of the batch is the state the marks describe: its decode (check: compare, the state was
// decoded the usual way too)
void launch_predecoded(const Work& w, uint32_t u, const PreMarks& m, bool check, hipStream_t s);

// ---- launch entry points (yc_decode.hip / yc_merge.hip / yc_encode.hip / yc_prims.hip)
void launch_chunks(const Work& w, hipStream_t s);  // k_spec + k_walk: large updates
void launch_direct(const Work& w, hipStream_t s);  // k_direct: small updates
bool wave_decode(const Work& w);                  // few small updates: k_wlen + k_wrank (else k_direct)
void launch_client_hash(const Work& w, uint64_t* key, uint32_t* val, uint32_t mask, hipStream_t s);
bool sections_small(const Work& w, uint32_t nsections, uint64_t* key, uint32_t* val, uint32_t mask, hipStream_t s);  // ranks + client table + hash, one workgroup
void launch_struct_count(const Work& w, hipStream_t s);
void launch_struct_scatter(const Work& w, hipStream_t s);
void launch_ds_bound(const Work& w, hipStream_t s);
bool count_ds_small(const Work& w, hipStream_t s);  // counts + delete-set bounds in one workgroup (small batches)
void launch_ds_decode(const Work& w, hipStream_t s);
void launch_section_clients(const Work& w, uint32_t nsections, hipStream_t s);
void launch_client_table(Work& w, uint32_t nsections, hipStream_t s);
void launch_struct_decode(const Work& w, uint32_t nstructs, hipStream_t s);
void launch_struct_lenscan(const Work& w, uint32_t nstructs, hipStream_t s);
bool decode_tail_small(const Work& w, uint32_t nstructs, uint32_t nsections, hipStream_t s);
void launch_decode_tail_small(const Work& w, uint32_t nstructs, uint32_t nsections, hipStream_t s);  // NONE: counts on the device  // one workgroup: structs .. client states (small, integrate)
void launch_json_structs(const Work& w, uint32_t nstructs, hipStream_t s);  // JSON.parse of JSON-like contents
// JSON.stringify(JSON.parse(.)) of the listed structs' contents (k_json_canon): one lane per struct,
// an arena of `acap` words per lane. pass 0 sizes them (items), pass 1 writes them at out + offs[j].
struct JItem {
  unsigned long long cpos;  // the content's first byte, as a batch-buffer position (window included)
  uint32_t clen;            // its bytes in the update
  uint32_t len;             // its canonical bytes
  uint32_t res;             // JSON_OK / JSON_BAD / JSON_ARENA
  uint32_t pad;             // pass 1: the canonical bytes differ from the input
};
void launch_json_canon(const Work& w, const uint32_t* list, uint32_t n, JItem* items, uint32_t* arena, uint32_t acap,
                       uint32_t lanes, const unsigned long long* offs, uint8_t* out, hipStream_t s);
void launch_states(const Work& w, uint32_t nstructs, uint32_t nsections, hipStream_t s);  // clocks + client states
void launch_struct_clocks(const Work& w, uint32_t nstructs, hipStream_t s);               // clocks only (lazy)

void launch_units_fill(const Work& w, uint64_t nunits, hipStream_t s);
void launch_units(const Work& w, uint32_t nstructs, uint32_t nclients, uint32_t nds, uint64_t nunits, bool ds_big, hipStream_t s);
constexpr uint32_t DSA_WAVE = 4096;  // delete-set ranges one wavefront applies per update (k_units); the rest spread
void launch_segments(const Work& w, uint32_t nclients, uint64_t nunits, hipStream_t s);
void launch_segment_props_fill(const Work& w, uint32_t nsegs, hipStream_t s);
void launch_segment_props(const Work& w, uint32_t nsegs, uint32_t nclients, uint64_t nunits, hipStream_t s);
uint32_t run_key_resolution(const Work& w, uint32_t nsegs, hipStream_t s);
uint32_t run_descent(const Work& w, uint32_t nsegs, hipStream_t s, bool fold_overwrite);
void launch_mapx_flip(const Work& w, uint32_t nsegs, hipStream_t s);  // full-YATA map entries -> the YATA kernels
void launch_mapx_fix(const Work& w, uint32_t nsegs, hipStream_t s);   // ... and back: the last one wins
bool merge_small_fits(uint64_t nsegs_bound);  // map-only small merges: one workgroup (k_merge_small)
void launch_merge_small(const Work& w, uint32_t nsegs, uint64_t nunits, hipStream_t s);  // nunits != 0: segments too, nsegs on the device
bool launch_merge_flags(const Work& w, uint32_t nsegs, hipStream_t s, bool fold_overwrite);  // true: run ids scanned too
bool encode_runs_small(uint32_t nsegs);  // the one-workgroup delete-set runs (k_runs_small)
void launch_merge_flags_only(const Work& w, uint32_t nsegs, hipStream_t s, bool fold_overwrite);
void launch_merge_tail(const Work& w, uint32_t nsegs, hipStream_t s);
// key-hash shards of one document (yc_merge.hip)
void launch_key_shards(const Work& w, uint32_t nsegs, uint32_t nshards, uint32_t* key_shard, uint8_t* owner, hipStream_t s);
void launch_shard_mask(const Work& w, uint32_t nsegs, const uint8_t* owner, uint32_t shard, hipStream_t s);
void launch_shard_export(const Work& w, uint32_t nsegs, const uint8_t* owner, uint32_t shard, uint32_t* acc, hipStream_t s);
void launch_merge_final(const Work& w, uint32_t nsegs, hipStream_t s);
void run_dead_keys(const Work& w, uint32_t nsegs, hipStream_t s);
constexpr uint32_t DS_TAIL_MIN = 4096, DS_TAILS_CAP = 1u << 16;  // long delete-set runs (yc_merge.hip k_ds_tails)
constexpr uint32_t DSP_MAXBLK = 8192;  // client blocks of one delete set decoded grid-wide (yc_decode.hip)
constexpr uint32_t DSH_STRIDE = 32, DSH_SEG = DSP_MAXBLK / DSH_STRIDE;  // header jumps (yc_decode.hip k_dsh_*)
constexpr uint32_t DSH_MIN_BLOCKS = 32;  // delete sets of more client blocks take the jumps
constexpr uint32_t LISTS_UNNUMBERED = 0xFFFFFFFFu;  // launch_yata: lists exist, launch_ylists numbers them
uint32_t launch_yata(const Work& w, uint32_t nsegs, uint32_t narray, uint32_t nclients, hipStream_t s, hipStream_t side,
                     hipEvent_t ev_fork, hipEvent_t ev_join);
uint32_t launch_ylists(const Work& w, uint32_t nsegs, hipStream_t s);

// side / ev_fork / ev_join / tmp2: the delete-set run chain runs on `side` with its own scan space
void launch_encode_sizes(const Work& w, uint32_t nsegs, uint32_t nclients, hipStream_t s, hipStream_t side,
                         hipEvent_t ev_fork, hipEvent_t ev_join, void* tmp2, size_t tmp2_bytes, bool runs_scanned);
void launch_out_sizes(const Work& w, uint32_t nsegs, uint32_t nclients, hipStream_t s);
void launch_encode_layout(const Work& w, uint32_t nsegs, uint32_t nclients, hipStream_t s, hipEvent_t ev_join);
void launch_encode_write(const Work& w, uint32_t nsegs, uint32_t nclients, hipStream_t s);
void launch_write_structs(const Work& w, uint32_t nsegs, uint32_t nclients, hipStream_t s);
bool encode_small_fits(uint64_t nsegs_bound, uint32_t nclients);  // the whole encode, one workgroup (small batches)
void launch_encode_small(const Work& w, uint32_t nsegs, uint32_t nclients, hipStream_t s);  // nsegs NONE: read on the device

// rocPRIM wrappers (yc_prims.hip)
size_t prim_tmp_bytes(uint64_t scan_n, uint64_t sort_n);  // scratch for scans of scan_n / sorts of sort_n items
void scan_u32(void* tmp, size_t tmpb, const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t s);          // exclusive
void scan_u32_to_u64(void* tmp, size_t tmpb, const uint32_t* in, uint64_t* out, uint64_t n, hipStream_t s);   // exclusive
void sort_u32(void* tmp, size_t tmpb, const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t s);
// device byte pieces: copy `len` bytes src -> dst, or (src == nullptr) write inl[0..len) (len <= 8)
struct Piece {
  const uint8_t* src;
  uint8_t* dst;
  uint32_t len;
  uint8_t inl[8];
};
void copy_pieces(const Piece* pieces, uint32_t n, hipStream_t s);
// per-document (lo, hi, n) of the struct / delete-set / state-vector sections of a multi-document encode
void launch_doc_ranges(const Work& w, uint32_t nclients, uint32_t ndocs, unsigned long long* rng, hipStream_t s);
// batched u32 fills (n in 32-bit words)
struct FillDesc { uint32_t* p; uint64_t n; uint32_t v; };
constexpr uint32_t FILL_MAX = 8;
struct FillBatch { FillDesc d[FILL_MAX]; uint32_t count; };
void fill_u32_multi(std::initializer_list<FillDesc> fills, hipStream_t s);
void sort_pairs_u32(void* tmp, size_t tmpb, const uint32_t* kin, uint32_t* kout, const uint32_t* vin, uint32_t* vout,
                    uint64_t n, hipStream_t s);
void sort_pairs_u64_u32(void* tmp, size_t tmpb, const uint64_t* kin, uint64_t* kout, const uint32_t* vin, uint32_t* vout,
                        uint64_t n, hipStream_t s, uint32_t end_bit = 64);  // (keys below 2^end_bit: fewer radix passes)
// inclusive scan with "max within equal high words" (segmented running max of packed values)
void scan_segmax_u64(void* tmp, size_t tmpb, const uint64_t* in, uint64_t* out, uint64_t n, hipStream_t s);

// lazy merge (yc_lazy.hip)
void launch_lazy_merge(Work& w, uint32_t nsections, uint32_t nclients, hipStream_t s);
void launch_lazy_merge_seq(Work& w, uint32_t cap_ev, uint32_t cap_blk, hipStream_t s);
void launch_lazy_diff(Work& w, uint32_t nsections, hipStream_t s);
uint32_t launch_event_sizes(Work& w, hipStream_t s, uint32_t* nslots_out);
uint32_t launch_ds_runs(Work& w, uint32_t nds, bool merge, hipStream_t s);
uint32_t launch_ds_write_sizes(Work& w, uint32_t nr, hipStream_t s);
void launch_lazy_write(Work& w, uint32_t nslots, uint32_t nr, uint32_t dsbase, hipStream_t s);

}  // namespace yc

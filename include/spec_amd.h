/*
 * spec_amd.h — C ABI of the MI355X bulk encode/decode engine for the spec binary format.
 *
 * This is the drop-in boundary for the reference's hot path (basecomplextech/spec,
 * encode.go / decode.go / writer*.go over internal/{encode,decode,format,writer,types}).
 * The reference has no batch API: callers loop over records calling
 * spec.OpenMessageErr + generated getters (decode) or NewMessageWriterBuffer + FieldWriter
 * calls + Build (encode).  Each entry point below replaces exactly such a loop over a
 * batch of records resident in HBM, with results identical to the per-record Go calls.
 * The Go binding a maintainer would add (cgo) is shown in INTEGRATION.md.
 *
 * Conventions
 *  - Plain C types only; all buffers are caller-owned DEVICE pointers unless a name ends
 *    in _host.  `stream` is a hipStream_t passed as void* (NULL = default stream).
 *  - Return value: SPEC_OK (0) or a negative SPEC_E_* code; launches are asynchronous.
 *  - A batch is `stream_bytes[stream_len]` = records concatenated, and
 *    `ends[n]` = exclusive end offset of each record (record i = [ends[i-1], ends[i]),
 *    ends[-1] = 0): the layout an mpx receiver produces after framing
 *    (mpx/conn_reader.go:179-194).  One call handles stream_len < 4 GiB; larger batches
 *    are split by the caller (string/bytes offsets are 32-bit, see below).
 *  - Columns are structure-of-arrays, one array per schema field, record-major, with the
 *    element width of spec_kind_width(kind).  string/bytes columns hold spec_span
 *    {uint32 off, uint32 len}: off is relative to the batch stream (decode output) or to
 *    the field's heap (encode input); an absent or empty value is {0, 0}.
 */
#ifndef SPEC_AMD_H
#define SPEC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version history (a binding compares spec_abi_version() with the header it was built against,
 * and spec_struct_size / spec_struct_offset with its own struct mirrors):
 *   1  rounds 1-4: SPEC_MAX_FIELDS 64, SPEC_TREE_MAX_FIELDS 256 (spec_schema 260 B, spec_tree 2052 B);
 *   2  SPEC_MAX_FIELDS / SPEC_NESTED_MAX_FIELDS / SPEC_TREE_MAX_FIELDS 1024: spec_schema 4100 B,
 *      spec_nested_schema.item at offset 4100, spec_tree 8196 B; spec_struct_size / _offset added;
 *      spec_lz4_state.reserved became content_checksum (same layout); spec_lz4_content added. */
#define SPEC_AMD_ABI_VERSION 2
/* Fields of a flat schema.  Schemas of up to 64 fields run the schema-specialised kernels; wider
 * ones decode in chunks of 64 fields (the generic kernel once per chunk, each getter against the
 * record's whole table) and encode through the wide kernels, whose field set the call writes into
 * the workspace.  A nested schema's halves hold up to 1024 fields each; when a half holds more
 * than 64, outer + item fields (the list field included) are at most SPEC_TREE_MAX_FIELDS, else
 * every nested entry point returns SPEC_E_INVALID_ARGUMENT: such a schema decodes in chunks of 64
 * fields per half and encodes through the schema-tree encoder, with its scratch allocated
 * stream-ordered by the call. */
#define SPEC_MAX_FIELDS 1024
#define SPEC_NESTED_MAX_FIELDS 1024

/* Column kinds: one per typed getter / FieldWriter method
 * (internal/types/msg.go:219-421, internal/writer/msg.go:99-211). */
typedef enum spec_kind {
    SPEC_KIND_BOOL = 1,    /* uint8 0/1        Message.Bool     / FieldWriter.Bool    */
    SPEC_KIND_BYTE = 2,    /* uint8            Message.Byte     / FieldWriter.Byte    */
    SPEC_KIND_INT16 = 3,   /* int16            Message.Int16    / FieldWriter.Int16   */
    SPEC_KIND_INT32 = 4,   /* int32            Message.Int32    / FieldWriter.Int32   */
    SPEC_KIND_INT64 = 5,   /* int64            Message.Int64    / FieldWriter.Int64   */
    SPEC_KIND_UINT16 = 6,  /* uint16           Message.Uint16   / FieldWriter.Uint16  */
    SPEC_KIND_UINT32 = 7,  /* uint32           Message.Uint32   / FieldWriter.Uint32  */
    SPEC_KIND_UINT64 = 8,  /* uint64           Message.Uint64   / FieldWriter.Uint64  */
    SPEC_KIND_FLOAT32 = 9, /* float32 bits     Message.Float32  / FieldWriter.Float32 */
    SPEC_KIND_FLOAT64 = 10,/* float64 bits     Message.Float64  / FieldWriter.Float64 */
    SPEC_KIND_BIN64 = 11,  /* 8 opaque bytes   Message.Bin64    / FieldWriter.Bin64   */
    SPEC_KIND_BIN128 = 12, /* 16 opaque bytes  Message.Bin128   / FieldWriter.Bin128  */
    SPEC_KIND_BIN256 = 13, /* 32 opaque bytes  Message.Bin256   / FieldWriter.Bin256  */
    SPEC_KIND_STRING = 14, /* spec_span        Message.String   / FieldWriter.String  */
    SPEC_KIND_BYTES = 15,  /* spec_span        Message.Bytes    / FieldWriter.Bytes   */
    SPEC_KIND_LIST = 16,   /* list<message> in spec_nested_schema.outer (its column is the item_begin CSR
                              index); in a spec_tree, a list of any element kind.
                                               Message.List / FieldWriter.List                    */
    SPEC_KIND_STRUCT = 17, /* spec_tree only: a generated struct (OpenXxx(FieldRaw) / EncodeXxxTo)   */
    SPEC_KIND_MESSAGE = 18,/* spec_tree only: a sub-message (Message(tag) / FieldWriter.Message)     */
    SPEC_KIND_ANY = 19,    /* spec_tree only: spec_span of the raw value (Field(tag) / Field(tag).Any) */
} spec_kind;

/* Per-record status: the error class OpenMessageErr returns for the record
 * (internal/decode/msg.go:14-99).  Field-level errors are swallowed by the getters,
 * which return zero values, exactly as in the reference. */
typedef enum spec_status {
    SPEC_STATUS_OK = 0,
    SPEC_STATUS_INVALID_TYPE = 1,       /* "decode message: invalid type"       */
    SPEC_STATUS_INVALID_TABLE_SIZE = 2, /* "decode message: invalid table size" */
    SPEC_STATUS_INVALID_DATA_SIZE = 3,  /* "decode message: invalid data size"  */
    SPEC_STATUS_INVALID_TABLE = 4,      /* "decode message: invalid table"      */
    SPEC_STATUS_INVALID_DATA = 5,       /* "decode message: invalid data"       */
    SPEC_STATUS_PANIC = 6,              /* the reference would panic (malformed list table) */
    SPEC_STATUS_INVALID_VALUE = 7,      /* spec_parse_messages: a nested value failed to parse */
    SPEC_STATUS_TOO_DEEP = 8,           /* spec_parse_messages: nesting deeper than 2,097,152 levels
                                           (the reference's recursion exhausts Go's 1 GB stack
                                           at a depth of that order) */
} spec_status;

typedef enum spec_rc {
    SPEC_OK = 0,
    SPEC_E_INVALID_ARGUMENT = -1,
    SPEC_E_HIP = -2,       /* a HIP runtime call failed (see spec_last_hip_error) */
    SPEC_E_TOO_LARGE = -3, /* stream_len >= 4 GiB or a record > format.MaxSize */
    SPEC_E_CAPACITY = -4,  /* output buffer smaller than the encoded batch */
    SPEC_E_WORKSPACE = -5, /* workspace smaller than *_workspace_size() */
    SPEC_E_CORRUPT = -6,   /* corrupt LZ4 frame (magic, version, header/block checksum, block size) */
    SPEC_E_ENCODE = -7,    /* an encoder error in some shard (a span outside its heap, a value > MaxSize) */
} spec_rc;

typedef struct spec_span {
    uint32_t off;
    uint32_t len;
} spec_span;

typedef struct spec_field {
    uint16_t tag;  /* message field tag (1..65535) */
    uint8_t kind;  /* spec_kind */
    uint8_t reserved;
} spec_field;

/* A flat message schema: the fields a generated Write() emits, in write order
 * (internal/lang/generator/message.go:319-439 emits one FieldWriter call per field). */
typedef struct spec_schema {
    uint32_t nfields;
    spec_field fields[SPEC_MAX_FIELDS];
} spec_schema;

/* A message with one list<message> field (BASELINE config 4, list_msg.go / writer_list_msg.go):
 * `outer` lists the outer message's fields in write order, exactly one of kind SPEC_KIND_LIST;
 * `item` the fields of each list item (flat kinds only). */
typedef struct spec_nested_schema {
    spec_schema outer;
    spec_schema item;
} spec_nested_schema;

/* ---- schema trees: every kind a generated reader/writer handles ----
 * A spec_tree describes a record message as fields in PRE-ORDER: each field names its enclosing
 * field (`parent`, an earlier index; -1 = the record).  Enclosing fields are
 *   SPEC_KIND_MESSAGE            its children are the sub-message's fields (write order);
 *   SPEC_KIND_STRUCT             its children are the struct's members in declaration order:
 *                                scalar kinds or other structs ("structs support only value
 *                                types or other structs", internal/lang/model/struct_field.go:
 *                                57-70), at most SPEC_TREE_MAX_STRUCT_DEPTH structs deep; a
 *                                struct is decoded members-last-first, an inner struct through its
 *                                own DecodeXxx, as generated Decode does
 *                                (internal/lang/generator/struct.go:75-113), and encoded members-
 *                                first then EncodeStruct (struct.go:115-142);
 *   SPEC_KIND_LIST, elem MESSAGE its children are the item message's fields;
 *   SPEC_KIND_LIST, elem STRUCT  its children are the struct's members (as above).
 * A list of scalars (elem = a scalar kind) has no children.  Enums are SPEC_KIND_INT32
 * (internal/lang/generator/enum.go:69-92).  Recursive types (pkg1.spec Submessage.next) are
 * unrolled to the depth the caller reads, exactly as a reader only opens what it accesses.
 *
 * Decoded output is a set of TABLES (spec_tree_layout): table 0 = the records; one table per
 * MESSAGE field (a row per row of its owner table: the sub-message of that row) and one per
 * LIST field (a row per list element, CSR-indexed by `begin` over its owner's rows).  Columns,
 * table by table, in this order:
 *   [BEGIN]  (LIST tables) uint32 [owner rows + 1]: row i's elements are [begin[i], begin[i+1])
 *   per direct field, in field order:
 *     scalar          VALUE  m.<Kind>(tag)                          (internal/types/msg.go:219-421)
 *     STRUCT          VALUE per scalar member, inner structs' members in place (pre-order):
 *                     OpenXxx(m.FieldRaw(tag))                       (msg.go:139-150)
 *     ANY             VALUE spec_span of m.Field(tag) = OpenValue   (msg.go:108-124, value.go:18-31),
 *                     then TYPE uint8 m.Field(tag).Type() (value.go:115-119: the value's last
 *                     byte, 0 for nil); Field(tag).<Kind>() / .Message(): spec_decode_values,
 *                     spec_tree_decoder_index_spans
 *     MESSAGE, LIST   PRESENT uint8 m.HasField(tag)                 (msg.go:101-106)
 *   a list of scalars: VALUE = ValueList.Get(i) (list_value.go:87-92); a list of structs: a
 *   VALUE per scalar member (pre-order);
 *   ERRMASK uint64 x W (MESSAGE-shaped tables: records, sub-messages, message-list items; W =
 *   ceil(direct fields / 64), at least 1: the column is 8 W bytes wide): bit k % 64 of word k / 64
 *   set when the k-th direct field's (write order) *Err getter errs — scalars
 *   <Kind>Err (msg.go:233-459), ANY OpenValueErr (value.go:35-46), MESSAGE MessageErr, LIST
 *   ListErr (msg.go:453-463), STRUCT DecodeXxx (generator/struct.go:60-64); an absent field never
 *   errs;
 *   STATUS uint8: records OpenMessageErr's class; sub-messages MessageErr's class (0 if absent);
 *   list items OpenItemErr's class or SPEC_STATUS_PANIC (Go panics: element start > end);
 *   list values / structs SPEC_STATUS_INVALID_VALUE when GetErr fails; any row whose struct or
 *   any field would make Go panic (slice out of range) SPEC_STATUS_PANIC.
 * Encode input uses the same columns (STATUS, ERRMASK, TYPE ignored): scalars and structs are always written,
 * MESSAGE / LIST fields when PRESENT is non-zero (a present list may be empty), ANY when its span
 * is non-empty (FieldWriter.Any copies the bytes: internal/writer/writer.go:438-456). */
#define SPEC_TREE_MAX_FIELDS 1024
#define SPEC_TREE_MAX_TABLES 128
#define SPEC_TREE_MAX_COLUMNS 2048
#define SPEC_TREE_MAX_DIRECT 1024 /* direct fields of one message / members of one struct (any, up to the tree's fields) */
#define SPEC_TREE_MAX_STRUCT_DEPTH 16 /* structs nested in structs (the outermost counts 1) */

typedef struct spec_tree_field {
    uint16_t tag;    /* field tag (ignored for struct members) */
    uint8_t kind;    /* spec_kind */
    uint8_t elem;    /* SPEC_KIND_LIST: element kind (a scalar kind, STRUCT or MESSAGE) */
    int16_t parent;  /* enclosing field, -1 = the record */
    uint16_t reserved;
} spec_tree_field;

typedef struct spec_tree {
    uint32_t nfields;
    spec_tree_field fields[SPEC_TREE_MAX_FIELDS];
} spec_tree;

typedef enum spec_tree_rel { SPEC_REL_ROOT = 0, SPEC_REL_ONE = 1, SPEC_REL_MANY = 2 } spec_tree_rel;
typedef enum spec_tree_shape { SPEC_SHAPE_MESSAGE = 0, SPEC_SHAPE_VALUE = 1, SPEC_SHAPE_STRUCT = 2 } spec_tree_shape;
typedef enum spec_tree_role {
    SPEC_COL_VALUE = 0, SPEC_COL_PRESENT = 1, SPEC_COL_BEGIN = 2, SPEC_COL_STATUS = 3,
    SPEC_COL_ERRMASK = 4, SPEC_COL_TYPE = 5
} spec_tree_role;

typedef struct spec_tree_table {
    int16_t parent;  /* owner table (-1 for the records) */
    int16_t field;   /* defining MESSAGE / LIST field (-1 for the records) */
    uint8_t rel;     /* spec_tree_rel */
    uint8_t shape;   /* spec_tree_shape */
    uint16_t first_column, ncolumns;
} spec_tree_table;

typedef struct spec_tree_column {
    uint16_t table;
    int16_t field;   /* the field (a struct member for struct columns); the table's field for BEGIN/STATUS */
    uint8_t role;    /* spec_tree_role */
    uint8_t kind;    /* VALUE: scalar kind or SPEC_KIND_ANY */
    uint16_t width;  /* bytes per row; a BEGIN column has owner rows + 1 entries */
} spec_tree_column;

/* Validate a tree and describe its tables and columns (arrays of SPEC_TREE_MAX_TABLES /
 * SPEC_TREE_MAX_COLUMNS entries).  SPEC_E_INVALID_ARGUMENT on an invalid tree. */
int spec_tree_layout(const spec_tree *tree, spec_tree_table *tables, uint32_t *ntables, spec_tree_column *columns,
                     uint32_t *ncolumns);

/* Decode: for every record, the generated reader's getters over the whole tree.  A decoder
 * owns its device workspace (grown on demand, on its device) and is used on one stream at a time.
 * The decode is one asynchronous pass (row counts of list tables stay on the device):
 *   spec_tree_decoder_index: the pass without columns, then the table row counts on the host
 *     (rows[ntables]; one synchronisation); it also sizes the list buffers for the batch;
 *   spec_tree_decoder_decode: the pass with columns (columns[c] sized by spec_tree_layout and
 *     rows; NULL skips a column), asynchronous; the batch must be the one indexed;
 *   spec_tree_decoder_run: the pass over a new batch with columns, asynchronous, no host
 *     synchronisation: rows_out (device, ntables uint64) receives the row counts, ~0 for a list
 *     table that outgrew the decoder's capacity for it or the caller's columns, and for every
 *     table below such a list (their rows beyond capacity are not decoded: index a batch of that
 *     shape first, or spec_tree_decoder_reserve).  col_rows (host, ntables; may be NULL) = the
 *     rows the caller's columns of each table hold (a BEGIN column holds its owner table's rows
 *     + 1 entries): rows are clamped to them, nothing is written past them (SPEC_E_CAPACITY if
 *     a record table's columns hold fewer than n rows).  With NULL, every list table's columns
 *     must hold spec_tree_decoder_capacity rows;
 *   spec_tree_decoder_capacity: the decoder's row capacity per list table (host; 0 for tables
 *     with a row per record);
 *   spec_tree_decoder_reserve: list-table capacities of at least rows[t] (host). */
typedef struct spec_tree_decoder spec_tree_decoder;
int spec_tree_decoder_create(const spec_tree *tree, spec_tree_decoder **out);
void spec_tree_decoder_destroy(spec_tree_decoder *d);
int spec_tree_decoder_index(spec_tree_decoder *d, const uint8_t *stream_bytes, uint64_t stream_len,
                            const uint64_t *ends, uint64_t n, uint64_t *rows, void *stream);
int spec_tree_decoder_decode(spec_tree_decoder *d, void *const *columns, void *stream);
int spec_tree_decoder_run(spec_tree_decoder *d, const uint8_t *stream_bytes, uint64_t stream_len, const uint64_t *ends,
                          uint64_t n, void *const *columns, const uint64_t *col_rows, uint64_t *rows_out,
                          void *stream);
int spec_tree_decoder_capacity(const spec_tree_decoder *d, uint64_t *rows);
int spec_tree_decoder_reserve(spec_tree_decoder *d, const uint64_t *rows);
/* spec_tree_jit_compile: compile (hiprtc, no GPU needed) the decoder's schema-specialised group
 * kernels for this tree into the code-object cache (a decoder compiles them on first use
 * otherwise); returns the code object's size, or <= 0 (SPEC_E_INVALID_ARGUMENT: invalid tree). */
long long spec_tree_jit_compile(const spec_tree *tree);
/* spec_tree_decoder_index over VALUE SPANS instead of contiguous records: row i of the root table
 * is the message spans[i] holds — what m.Field(tag).Message() opens (an `any` / `message` field,
 * internal/lang/generator/message.go:145-148; Value.Message() = OpenMessage,
 * internal/types/value.go:318-321).  A nil span is an empty message; a span past the stream
 * is a Go panic (STATUS SPEC_STATUS_PANIC).  Decode with spec_tree_decoder_decode as usual. */
int spec_tree_decoder_index_spans(spec_tree_decoder *d, const uint8_t *stream_bytes, uint64_t stream_len,
                                  const spec_span *spans, uint64_t n, uint64_t *rows, void *stream);

/* Value.<Kind>() / Value.<Kind>Err() (internal/types/value.go:120-310) over n value spans (an
 * `any` column): out[i] = Decode<Kind>(the span's bytes) (n * spec_kind_width(kind) bytes;
 * string/bytes as spans into the stream), err[i] (optional) = 1 where the decoder errs, 2 where
 * the span lies past the stream (Go would panic), else 0. */
int spec_decode_values(int kind, const uint8_t *stream_bytes, uint64_t stream_len, const spec_span *spans, uint64_t n,
                       void *out, uint8_t *err, void *stream);

/* Encode: for every record, the generated Write() over the tree, Build() (writer.go:141-188),
 * appended into out[] with ends[i] = record i's end.  rows[t] = rows of table t (host);
 * heaps[c] / heap_lens[c] back string, bytes and any columns (NULL otherwise).  Writes *total
 * (device); if it exceeds out_cap nothing is written; an encoder error (a span outside its heap,
 * a value > format.MaxSize, a BEGIN column not monotonic) makes *total all-ones.  With
 * out == NULL only *total is computed.  Workspace: spec_encode_tree_workspace_size(tree, rows). */
size_t spec_encode_tree_workspace_size(const spec_tree *tree, const uint64_t *rows);
int spec_encode_tree(const spec_tree *tree, const void *const *columns, const uint8_t *const *heaps,
                     const uint64_t *heap_lens, const uint64_t *rows, uint8_t *out, uint64_t out_cap, uint64_t *ends,
                     void *workspace, size_t workspace_size, uint64_t *total, void *stream);

/* ---- several devices in one process (the reference has no multi-device code) ----
 * Records are independent, so a batch splits into contiguous record shards, one per device.  A
 * spec_shard holds per device a stream and, with more than one device (or SPEC_SHARD_FORCE_COMM),
 * an RCCL communicator rank (ncclCommInitAll over the listed devices, no duplicates; librccl is
 * loaded on first use).  Per device, a shard decodes into ONE packed buffer: the schema's
 * columns back to back, each starting on a 256-byte boundary, then the status bytes
 * (spec_packed_layout; what spec_amd.shard.PackedColumns lays out), so the gather to the root
 * device is one grouped RCCL send/recv per device over xGMI.  String/bytes spans stay
 * shard-relative (a 16M-record batch is > 4 GiB): the shard's byte base travels alongside.
 * Every call replaces the per-record loop of decode.go:9-40 / internal/types/msg.go:43-55
 * (decode) or internal/writer/writer.go:520-553 -> internal/encode/msg.go:15-77 (encode) over
 * the shard, exactly as spec_decode_flat / spec_encode_flat do on one device.
 *   spec_packed_layout: column offsets / status offset of n records; returns the bytes;
 *   spec_shard_bounds: shard k's records [r0, r1) of n (sizes differ by at most one);
 *   spec_shard_bounds_bytes: shard k's records [r0, r1) of n such that the shards' BYTES are
 *     near-equal: `ends` is any non-decreasing cumulative byte count per record (a batch's end
 *     offsets; for encode, e.g. a prefix sum of the records' heap bytes), split point k the
 *     record boundary nearest to ends[n-1] * k / nshards (binary search).  Records are
 *     variable-length (internal/encode/bytes.go:14-26, string.go:14-26), so with skewed sizes
 *     a record split leaves the slowest device with most of the bytes;
 *   spec_shard_set_split: how spec_shard_decode_host and spec_shard_host_decode split a host
 *     batch: SPEC_SHARD_SPLIT_RECORDS (default, spec_shard_bounds) or SPEC_SHARD_SPLIT_BYTES
 *     (spec_shard_bounds_bytes over the batch's ends);
 *   spec_shard_create_ex: flags SPEC_SHARD_FORCE_COMM = build the communicator even for one
 *     device; the gather then moves every part, the root's own too, through RCCL;
 *     SPEC_SHARD_SHARED = devices may repeat (several shards on one GPU, no communicator, the
 *     gather is device copies): the multi-shard flow on a machine with fewer GPUs;
 *   spec_shard_has_comm: 1 when the communicator exists; spec_shard_rccl_version: ncclGetVersion
 *     of the RCCL in use (< 0 if none loads);
 *   spec_shard_decode: device i decodes its device-resident shard (streams[i], ends[i] relative
 *     to streams[i], ns[i] records) into packed[i] (on device i), asynchronously on its stream;
 *   spec_shard_decode_host: a host batch split by the shard's split mode; per device, on its own host
 *     thread, the shard is copied in spec_shard_set_chunks record chunks (default 8; through
 *     pinned staging slots when the batch is pageable) and every chunk decoded once it has
 *     landed (ends rebased on the device); byte_bases[i] (optional) = shard i's first byte.
 *     Returns once every copy is issued; a pinned batch must stay valid until spec_shard_sync.
 *     Calls may follow each other without spec_shard_sync: a call's copies into the device's
 *     staging buffer are ordered after the previous call's decodes that read it;
 *   spec_shard_gather: every device's packed buffer (nbytes[i]) to `gathered` on device `root`,
 *     part i at the sum of the earlier parts' sizes, ordered after the decodes on each stream;
 *   spec_shard_encode: device i encodes its ns[i] records from columns[i] (heaps[i], heap_lens[i]
 *     as spec_encode_flat) into outs[i] (out_caps[i] bytes) with ends[i][r] = the record's end
 *     in the WHOLE batch: every device's size and write passes (the write pass needs no base: a
 *     record's bytes do not depend on its offset), one host wait for the size passes alone, the
 *     exclusive scan of the shard totals (byte_bases, host) while the writes run, then each
 *     shard's ends moved by its base.  totals[i] (host) = shard i's bytes (all-ones on an
 *     encoder error).  outs[0..ndev) back to back (e.g. through spec_shard_gather with nbytes =
 *     totals) are exactly one spec_encode_flat of the batch.  Each shard behaves as its own
 *     spec_encode_flat: one whose total exceeds its capacity or errs writes nothing; the call
 *     then returns SPEC_E_CAPACITY / SPEC_E_ENCODE and moves no ends to the whole batch (the
 *     shards that fit hold shard-relative ends).  Asynchronous after the size passes;
 *   spec_shard_stream: device k's stream; spec_shard_sync: wait for every device's streams.
 * A spec_shard is driven by one host thread at a time (it starts its own per-device threads). */
#define SPEC_SHARD_MAX_DEVICES 16
#define SPEC_SHARD_FORCE_COMM 1u
#define SPEC_SHARD_SHARED 2u
#define SPEC_SHARD_SPLIT_RECORDS 0u
#define SPEC_SHARD_SPLIT_BYTES 1u
typedef struct spec_shard spec_shard;
uint64_t spec_packed_layout(const spec_schema *schema, uint64_t n, uint64_t *col_offsets, uint64_t *status_offset);
void spec_shard_bounds(uint64_t n, int nshards, int k, uint64_t *r0, uint64_t *r1);
void spec_shard_bounds_bytes(const uint64_t *ends, uint64_t n, int nshards, int k, uint64_t *r0, uint64_t *r1);
int spec_shard_set_split(spec_shard *c, uint32_t split);
int spec_shard_create(const int *devices, int ndev, spec_shard **out);
int spec_shard_create_ex(const int *devices, int ndev, uint32_t flags, spec_shard **out);
void spec_shard_destroy(spec_shard *c);
int spec_shard_ndev(const spec_shard *c);
int spec_shard_has_comm(const spec_shard *c);
int spec_shard_rccl_version(void);
int spec_shard_set_chunks(spec_shard *c, uint32_t chunks);
void *spec_shard_stream(const spec_shard *c, int k);
int spec_shard_decode(spec_shard *c, const spec_schema *schema, const uint8_t *const *streams,
                      const uint64_t *stream_lens, const uint64_t *const *ends, const uint64_t *ns,
                      uint8_t *const *packed);
int spec_shard_decode_host(spec_shard *c, const spec_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                           const uint64_t *ends, uint64_t n, uint8_t *const *packed, uint64_t *byte_bases);
int spec_shard_gather(spec_shard *c, const uint64_t *nbytes, uint8_t *const *packed, int root, uint8_t *gathered);
int spec_shard_encode(spec_shard *c, const spec_schema *schema, const void *const *const *columns,
                      const uint8_t *const *const *heaps, const uint64_t *const *heap_lens, const uint64_t *ns,
                      uint8_t *const *outs, const uint64_t *out_caps, uint64_t *const *ends, uint64_t *totals,
                      uint64_t *byte_bases);
int spec_shard_sync(spec_shard *c);

/* ---- introspection ----
 * spec_abi_version: SPEC_AMD_ABI_VERSION of the library (a binding refuses to run on a mismatch).
 * spec_struct_size(which): sizeof the struct as the library was built (0 for an unknown id);
 * spec_struct_offset(which, member): offsetof its member-th member in declaration order
 * ((size_t)-1 past the last member or for an unknown id).  A binding that mirrors these structs
 * (cgo, ctypes) checks its own layout against them once at load time. */
typedef enum spec_abi_struct {
    SPEC_ABI_SPAN = 0,          /* spec_span {off, len} */
    SPEC_ABI_FIELD = 1,         /* spec_field {tag, kind, reserved} */
    SPEC_ABI_SCHEMA = 2,        /* spec_schema {nfields, fields} */
    SPEC_ABI_NESTED_SCHEMA = 3, /* spec_nested_schema {outer, item} */
    SPEC_ABI_TREE_FIELD = 4,    /* spec_tree_field {tag, kind, elem, parent, reserved} */
    SPEC_ABI_TREE = 5,          /* spec_tree {nfields, fields} */
    SPEC_ABI_TREE_TABLE = 6,    /* spec_tree_table {parent, field, rel, shape, first_column, ncolumns} */
    SPEC_ABI_TREE_COLUMN = 7,   /* spec_tree_column {table, field, role, kind, width} */
    SPEC_ABI_LZ4_BLOCK = 8,     /* spec_lz4_block {src_off, src_len, stored} */
    SPEC_ABI_LZ4_STATE = 9,     /* spec_lz4_state {in_frame, block_max, flags, content_checksum} */
    SPEC_ABI_LZ4_CONTENT = 10,  /* spec_lz4_content {v, total, buf, buffered, started} */
    SPEC_ABI_NSTRUCTS = 11
} spec_abi_struct;
int spec_abi_version(void);
size_t spec_struct_size(int which);
size_t spec_struct_offset(int which, int member);
int spec_kind_width(int kind);
const char *spec_strerror(int rc);
int spec_last_hip_error(void);

/* ---- memory and streams ----
 * Thin wrappers so a binding (cgo) needs only this header: device buffers,
 * pinned host staging (hipHostMalloc; Go code sees it through unsafe.Slice and never hands Go
 * memory to the device), streams and async copies.  All return SPEC_OK or SPEC_E_HIP. */
int spec_set_device(int device);
int spec_device_alloc(size_t bytes, void **ptr);
int spec_device_free(void *ptr);
int spec_host_alloc(size_t bytes, void **ptr);
int spec_host_free(void *ptr);
int spec_stream_create(void **stream);
int spec_stream_destroy(void *stream);
int spec_stream_sync(void *stream);
int spec_copy_h2d(void *dst, const void *src, size_t bytes, void *stream);
int spec_copy_d2h(void *dst, const void *src, size_t bytes, void *stream);
int spec_copy_d2d(void *dst, const void *src, size_t bytes, void *stream);

/* ---- decode ----
 * spec_decode_flat: for every record i, exactly
 *     m, err := spec.OpenMessageErr(record_i)          (msg.go:25-27, internal/types/msg.go:43-55)
 *     status[i] = class(err); column_f[i] = m.<Kind_f>(tag_f)   (internal/types/msg.go:219-475)
 * replacing the BenchmarkReadMessage loop (internal/bench/parse_test.go:48-111) and the
 * decoders it reaches (decode.go:9-40 -> internal/decode/...).
 * columns[f] points at n * spec_kind_width(kind_f) bytes; status may be NULL. */
int spec_decode_flat(const spec_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                     const uint64_t *ends, uint64_t n, void *const *columns, uint8_t *status,
                     void *stream);

/* spec_decode_flat_errors: spec_decode_flat plus, per record, which getters' *Err variants
 * return an error (internal/types/msg.go:233-459: Int32Err, StringErr, ...): errmask[i] bit f
 * is set when field f is present and Decode<Kind> fails on it (an absent field is no error;
 * the record-level OpenMessageErr class is in status).  A schema of more than 64 fields has
 * ceil(nfields / 64) mask words per record, word-major: errmask[c * n + i] bit f is field
 * 64 c + f of record i.
 * Runs the schema-specialised kernel's errmask variant where the schema has one (else the
 * generic kernel): the same columns and status as spec_decode_flat. */
int spec_decode_flat_errors(const spec_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                            const uint64_t *ends, uint64_t n, void *const *columns, uint8_t *status, uint64_t *errmask,
                            void *stream);

/* spec_decode_flat_range: records [r0, r1) of a batch only — stream_bytes/stream_len/ends
 * describe the WHOLE batch (absolute offsets) and columns/status are indexed by record, so a
 * host pipeline can decode chunk k while chunk k+1 is still being copied in.  range_bytes =
 * bytes the range spans (sizes the per-wave LDS staging; 0 = use stream_len / r1). */
int spec_decode_flat_range(const spec_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                           const uint64_t *ends, uint64_t r0, uint64_t r1, uint64_t range_bytes, void *const *columns,
                           uint8_t *status, void *stream);

/* ---- mpx frames (the path's source: mpx/conn_reader.go:179-194, conn_writer.go:84-97) ----
 * An mpx connection carries frames [u32 big-endian size][message], back to back.
 * spec_frames_index (HOST memory, CPU): walks the heads of buf[0, len) and writes ends[k] =
 * offset just past frame k's message, for every complete frame (at most cap; SPEC_E_CAPACITY
 * if more remain); *count = frames indexed, *consumed = bytes they span (an incomplete tail
 * frame is left for the next read).
 * spec_decode_frames: spec_decode_flat_range over the frames in place (each record starts 4
 * bytes after the previous frame's end): no host-side compaction of the received bytes. */
int spec_frames_index(const uint8_t *buf, uint64_t len, uint64_t *ends, uint64_t cap, uint64_t *count,
                      uint64_t *consumed);
int spec_decode_frames(const spec_schema *schema, const uint8_t *frames, uint64_t frames_len,
                       const uint64_t *ends, uint64_t r0, uint64_t r1, uint64_t range_bytes, void *const *columns,
                       uint8_t *status, void *stream);
/* spec_frames_index_device: spec_frames_index on a DEVICE buffer (4-byte aligned), with the same
 * results: ends[0, min(frames, cap)), *count, *consumed (device uint64) and *status (device int32:
 * SPEC_OK, or SPEC_E_CAPACITY when more than cap complete frames exist — then *count = cap).  The
 * serial head chain is resolved in parallel: per 64 KiB segment the exit of every entry offset
 * below 2048, composed over groups of segments; a frame straddling a segment boundary by 2048
 * bytes or more (or > 4096 frames in a segment) falls back to a serial walk on the device.
 * Workspace: spec_frames_index_device_workspace_size(len) bytes.  Asynchronous on `stream`. */
size_t spec_frames_index_device_workspace_size(uint64_t len);
int spec_frames_index_device(const uint8_t *buf, uint64_t len, uint64_t *ends, uint64_t cap, uint64_t *count,
                             uint64_t *consumed, int32_t *status, void *workspace, size_t workspace_size,
                             void *stream);

/* ---- LZ4 (mpx connection compression: mpx/conn_writer.go:42-56, conn_reader.go:53-62) ----
 * mpx wraps a connection in ONE LZ4 frame of independent blocks (pierrec/lz4/v4, 256 KiB blocks).
 * spec_lz4_frame_blocks (HOST, CPU): walks the frame headers and block size words of buf[0, len)
 * (one u32 per block; header checksums, and block checksums when the frame has them, verified)
 * and lists every COMPLETE block; `state` carries an open frame across calls (zero it for a
 * new connection): a later call continues with the frame's blocks.  *consumed = bytes the listed
 * blocks (and finished frames) span.  SPEC_E_CORRUPT on a bad header, SPEC_E_CAPACITY when more
 * than cap blocks are complete.  When a frame that carries a content checksum ends in the call
 * (its end mark), state->flags bit 2 is set and state->content_checksum holds the stored
 * checksum: compare it with spec_lz4_content_digest over the frame's decompressed bytes (what
 * lz4.Reader checks at the frame's end, pierrec/lz4/v4 frame.go; mpx writes it when a connection
 * closes).
 * spec_lz4_decompress (DEVICE): block k (src[blocks[k].src_off, +src_len)) decompressed into
 * slots + k * slot_bytes (slot_bytes >= the block max size, a multiple of 16; slots 16-byte aligned); sizes[k] = its size, or
 * all-ones and status[k] = 1 for a corrupt block (pierrec decodeBlock's errors).
 * spec_lz4_pack (DEVICE): the slots gathered into out back to back; *total (device) = bytes,
 * all-ones if any block was corrupt; nothing written if *total > out_cap. */
typedef struct spec_lz4_block {
    uint64_t src_off; /* block data in the source buffer */
    uint32_t src_len;
    uint32_t stored;  /* 1: stored uncompressed (size word bit 31) */
} spec_lz4_block;
typedef struct spec_lz4_state {
    uint32_t in_frame;  /* 1: the next bytes continue an open frame's blocks */
    uint32_t block_max; /* that frame's block max size */
    uint32_t flags;     /* bit 0 block checksums, bit 1 content checksum; bit 2 (output): a frame
                           with a content checksum ended in this call */
    uint32_t content_checksum; /* with flags bit 2: that frame's stored content checksum */
} spec_lz4_state;
int spec_lz4_frame_blocks(const uint8_t *buf, uint64_t len, spec_lz4_state *state, spec_lz4_block *blocks,
                          uint64_t cap, uint64_t *nblocks, uint64_t *consumed, uint32_t *block_max);
int spec_lz4_decompress(const uint8_t *src, uint64_t src_len, const spec_lz4_block *blocks, uint64_t nblocks,
                        uint8_t *slots, uint64_t slot_bytes, uint32_t *sizes, uint8_t *status, void *stream);
size_t spec_lz4_pack_workspace_size(uint64_t nblocks);
int spec_lz4_pack(const uint8_t *slots, uint64_t slot_bytes, const uint32_t *sizes, uint64_t nblocks, uint8_t *out,
                  uint64_t out_cap, uint64_t *total, void *workspace, size_t workspace_size, void *stream);
/* The frame's content checksum on the DEVICE: xxHash32 (seed 0) of every byte the frame
 * decompresses to, streamed over any number of calls.  `content` is a DEVICE spec_lz4_content,
 * all zero for a new frame (hipMemset); spec_lz4_content_update appends data[0, len) (device, any
 * alignment), spec_lz4_content_digest writes the checksum of everything appended so far to
 * *digest (device uint32).  Asynchronous.  xxHash32 is serial over 16-byte stripes (four
 * accumulators): one wave's four lanes run it, a few GB/s — a check at the frame's end, not a
 * stage of the block pipeline. */
typedef struct spec_lz4_content {
    uint32_t v[4];      /* the four accumulators */
    uint64_t total;     /* bytes appended */
    uint8_t buf[16];    /* a partial stripe */
    uint32_t buffered;  /* bytes in buf */
    uint32_t started;   /* 0: fresh (zeroed) state */
} spec_lz4_content;
int spec_lz4_content_update(spec_lz4_content *content, const uint8_t *data, uint64_t len, void *stream);
int spec_lz4_content_digest(const spec_lz4_content *content, uint32_t *digest, void *stream);

/* ---- host pipeline (the path starts and ends in HOST memory: mpx connection buffers) ----
 * spec_host_decoder decodes a batch held in pinned host memory (spec_host_alloc) into a pinned
 * host output buffer, overlapping on three HIP streams the H2D copy of chunk k+1, the decode
 * of chunk k (spec_decode_flat_range) and the D2H copy of chunk k-1 — the receive loop of
 * mpx/conn_reader.go:179-194 followed by the per-record OpenMessageErr + getters, batched.
 * Outputs are CHUNK-MAJOR: chunk k (records [r0, r1) = [n*k/chunks, n*(k+1)/chunks)) is one
 * region of out_host — its records' column 0, column 1, ..., then their status bytes — so
 * each chunk leaves the device in one copy; spec_host_decoder_chunk gives the offsets.
 * Device buffers and streams are created once (n_cap records, stream_cap bytes);
 * spec_host_decoder_run is synchronous (returns when out_host is complete). */
typedef struct spec_host_decoder spec_host_decoder;
int spec_host_decoder_create(const spec_schema *schema, uint64_t n_cap, uint64_t stream_cap, uint32_t chunks,
                             spec_host_decoder **out);
void spec_host_decoder_destroy(spec_host_decoder *d);
uint64_t spec_host_decoder_out_bytes(const spec_host_decoder *d, uint64_t n);
int spec_host_decoder_chunk(const spec_host_decoder *d, uint64_t n, uint32_t k, uint64_t *r0, uint64_t *r1,
                            uint64_t *col_offsets, uint64_t *status_offset);
int spec_host_decoder_run(spec_host_decoder *d, const uint8_t *stream_host, uint64_t stream_len,
                          const uint64_t *ends_host, uint64_t n, uint8_t *out_host);

/* The host pipeline on every device of a spec_shard at once (host batch in, host columns out,
 * one host thread per device): spec_shard_host_prepare creates a spec_host_decoder per device
 * (n_cap / stream_cap per SHARD); spec_shard_host_decode splits the batch by the split mode
 * and runs device i's decoder over shard i into out_host[i] (that decoder's chunk-major layout:
 * spec_host_decoder_out_bytes / _chunk on spec_shard_host_decoder(c, i)), spans shard-relative,
 * byte_bases[i] (optional) = shard i's first byte.  Synchronous. */
int spec_shard_host_prepare(spec_shard *c, const spec_schema *schema, uint64_t n_cap, uint64_t stream_cap,
                            uint32_t chunks);
spec_host_decoder *spec_shard_host_decoder(const spec_shard *c, int k);
int spec_shard_host_decode(spec_shard *c, const uint8_t *stream_host, uint64_t stream_len, const uint64_t *ends_host,
                           uint64_t n, uint8_t *const *out_host, uint64_t *byte_bases);

/* ---- recursive validation ----
 * spec_parse_messages: for every record, spec.ParseMessage (msg.go:29-32 ->
 * internal/types/msg.go:58-82): the message table, then ParseValue on every non-empty field,
 * recursing into lists and messages (internal/types/list.go:35-53, value.go:49-113) — what
 * mpx runs on each received frame (mpx/conn_reader.go:119).  status[i]: SPEC_STATUS_OK, the
 * top-level trailer class (1-5), SPEC_STATUS_PANIC (a list element whose start > end: Go
 * panics), SPEC_STATUS_INVALID_VALUE (any nested error), or SPEC_STATUS_TOO_DEEP (more than
 * 2,097,152 nested containers: records deeper than 32 are parsed again with their stacks in a
 * stream-ordered HBM scratch of the call, 64 MiB).  sizes[i] (optional) =
 * ParseMessage's size (bytes of the message), 0 on error.  head = bytes before each record
 * (4 for mpx frames, see spec_frames_index). */
int spec_parse_messages(const uint8_t *stream_bytes, uint64_t stream_len, const uint64_t *ends, uint64_t n,
                        uint32_t head, uint8_t *status, uint32_t *sizes, void *stream);

/* spec_parse_batch: the same recursive validation from another root, per record:
 *   SPEC_PARSE_MESSAGE  spec.ParseMessage (= spec_parse_messages);
 *   SPEC_PARSE_LIST     spec.ParseList (list.go:26-29 -> internal/types/list.go:35-53): the list
 *                       table (its error class, 1-5), then ParseValue on every non-empty element;
 *                       an empty record is an empty list;
 *   SPEC_PARSE_VALUE    spec.ParseValue (value.go:30-33 -> internal/types/value.go:49-113): the
 *                       value's type (its last byte), its decoder's checks, lists and messages
 *                       recursively; any error SPEC_STATUS_INVALID_VALUE (an empty record:
 *                       "unsupported type 0").
 * A value whose size exceeds its slice (DecodeStruct does not bound its data size) makes
 * value.go:110's b[len(b)-n:] panic: SPEC_STATUS_PANIC, at any depth.  sizes[i] = the parsed
 * size (ParseValue's n; the bytes of the list / message). */
#define SPEC_PARSE_MESSAGE 0u
#define SPEC_PARSE_LIST 1u
#define SPEC_PARSE_VALUE 2u
int spec_parse_batch(uint32_t root, const uint8_t *stream_bytes, uint64_t stream_len, const uint64_t *ends, uint64_t n,
                     uint32_t head, uint8_t *status, uint32_t *sizes, void *stream);

/* spec_decode_flat_prepare: compile (once per device, schema and record-size class) the
 * schema-specialised decode kernel that spec_decode_flat uses when one exists — the
 * analogue of the reference's generated readers (internal/lang/generator/message.go:97-186).
 * Optional: spec_decode_flat compiles it on first use.  Returns 1 if a specialised kernel
 * is ready, 0 if the generic kernel will be used (schema without a fast path, JIT disabled
 * or unavailable), <0 on an invalid schema.  Results never differ between the two. */
int spec_decode_flat_prepare(const spec_schema *schema, uint64_t stream_len, uint64_t n);
/* spec_decode_flat_jit_compile: diagnostic — run only the hiprtc compile of that kernel
 * (no device needed); returns the code-object size, 0 if the schema has no fast path. */
long long spec_decode_flat_jit_compile(const spec_schema *schema, uint64_t stream_len, uint64_t n);
/* spec_encode_flat_jit_compile: diagnostic — the hiprtc compile of the schema-specialised
 * encode kernels spec_encode_flat_size/spec_encode_flat use (analogue of the generated
 * Write(), internal/lang/generator/message.go:319-439); code-object size, 0 if the schema
 * has none (list fields, more than 32 fields). */
long long spec_encode_flat_jit_compile(const spec_schema *schema);
/* spec_set_jit: 0 forces the generic kernel (also: environment SPEC_AMD_JIT=0). */
void spec_set_jit(int enabled);

/* ---- nested decode (list<message>) ----
 * For every record i, exactly what a generated reader does:
 *     m, err := spec.OpenMessageErr(record_i); status[i] = class(err); outer getters as above
 *     items := spec.NewMessageList(m.msg.List(list_tag), OpenItemErr)     list_msg.go:20-26,
 *                                                      internal/types/msg.go:441-444
 *     for j < items.Len(): item = items.Get(j) -> item getters             list_msg.go:88-92
 * Items are stored in record order: record i's items are [item_begin[i], item_begin[i+1]).
 * item_status[k] = class(OpenItemErr error), or SPEC_STATUS_PANIC where Go's
 * List.GetBytes would panic (element start > end, internal/types/list.go:100-116).
 * Two calls on the same workspace (spec_decode_nested_workspace_size(n) bytes):
 *   spec_decode_nested_index  -> *total_items (device uint64): size the item columns,
 *   spec_decode_nested        -> all columns; items beyond item_cap are not written.
 * outer_columns[f] for the SPEC_KIND_LIST field is ignored (may be NULL). */
size_t spec_decode_nested_workspace_size(uint64_t n);
int spec_decode_nested_index(const spec_nested_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                             const uint64_t *ends, uint64_t n, void *workspace, size_t workspace_size,
                             uint64_t *total_items, void *stream);
int spec_decode_nested(const spec_nested_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                       const uint64_t *ends, uint64_t n, void *const *outer_columns, uint8_t *status,
                       uint32_t *item_begin, void *const *item_columns, uint8_t *item_status, uint64_t item_cap,
                       void *workspace, size_t workspace_size, void *stream);
/* spec_decode_nested_onepass: the same outputs from ONE call, with no host round trip for the
 * item total: the index kernels and the decode kernel back to back on the stream (a library
 * built with -DSPEC_AB_LOOKBACK=1 runs one kernel instead, in which each 64-record group
 * publishes its item count and finds its first item by looking back over the groups before it).
 * Writes *total_items (device uint64); items at index >= item_cap are not
 * written — if *total_items > item_cap, call again with item columns of that size (the stream
 * bytes bound it: every item has a list-table entry of at least 2 bytes, so stream_len / 2
 * always suffices).
 * Same workspace size as spec_decode_nested; its contents are overwritten. */
int spec_decode_nested_onepass(const spec_nested_schema *schema, const uint8_t *stream_bytes, uint64_t stream_len,
                               const uint64_t *ends, uint64_t n, void *const *outer_columns, uint8_t *status,
                               uint32_t *item_begin, void *const *item_columns, uint8_t *item_status,
                               uint64_t item_cap, void *workspace, size_t workspace_size, uint64_t *total_items,
                               void *stream);
/* spec_set_nested_mode: the kernels of spec_decode_nested_index / spec_decode_nested (results
 * never differ; times per 1M config-4 records, index + decode):
 * 5 (default) as 4, the decode pass's blocks in XCD-aware order (neighbouring groups, which share
 *   the item columns' cache lines, on one XCD's L2: 0.127 ms, 1 % under 4);
 * 4 count pass from each record's last 64 bytes, decode with items found by an owner search over
 *   the group's record prefix sums (0.128 ms);
 * 1 count pass over the staged 64-record span, decode as 4 (0.140 ms);
 * 2 as 1, items read from ranges their records' lanes precomputed into LDS (0.141 ms);
 * 3 as 1 with LDS slabs for half a group (0.160 ms). */
void spec_set_nested_mode(int mode);
/* spec_decode_nested_jit_compile: compile (hiprtc, no GPU needed) the schema-specialised one-pass
 * kernel; code-object size, 0 if neither schema has a fast path. */
long long spec_decode_nested_jit_compile(const spec_nested_schema *schema);

/* ---- encode ----
 * spec_encode_flat: for every record i, exactly
 *     w := spec.NewMessageWriterBuffer(buf)             (writer_msg.go:26-31)
 *     w.Field(tag_f).<Kind_f>(column_f[i])  for f in schema order   (internal/writer/msg.go:99-211)
 *     w.Build()                                          (internal/writer/msg.go:56-60)
 * appending into one output buffer (encode.go:11-38 -> internal/encode/...), so out[] holds
 * the records back to back and ends[i] is each record's end offset.  heaps[f] (with
 * heap_lens[f] bytes) backs string/bytes column f; NULL for other kinds.
 * Needs a workspace of spec_encode_flat_workspace_size(n) bytes; writes the total encoded
 * size to *total (device uint64).  If the total exceeds out_cap, nothing is written to
 * out/ends and *total still reports the required size (check it, then retry).
 * spec_encode_flat_size runs only the sizing passes (writes *total). */
size_t spec_encode_flat_workspace_size(uint64_t n);
int spec_encode_flat_size(const spec_schema *schema, const void *const *columns, uint64_t n,
                          void *workspace, size_t workspace_size, uint64_t *total, void *stream);
int spec_encode_flat(const spec_schema *schema, const void *const *columns,
                     const uint8_t *const *heaps, const uint64_t *heap_lens, uint64_t n,
                     uint8_t *out, uint64_t out_cap, uint64_t *ends, void *workspace,
                     size_t workspace_size, uint64_t *total, void *stream);

/* ---- nested encode (list<message>) ----
 * For every record i, what a generated Write() does (writer_list_msg.go:8-47): the outer
 * fields in write order; at the SPEC_KIND_LIST field, w.Field(tag).List(), then for each
 * item k in [item_begin[i], item_begin[i+1]) l.Add() + the item fields + End(); l.End();
 * finally Build().  Items come from item_columns (nitems rows); string/bytes columns index
 * the matching heaps.  Writes out[], ends[] and *total (device); with out == NULL only
 * *total is computed.  If the total exceeds out_cap nothing is written; an encoder error
 * (string/bytes > MaxSize or outside its heap, item_begin not monotonic or > nitems) makes
 * *total all-ones.  Workspace: spec_encode_nested_workspace_size(n) bytes. */
size_t spec_encode_nested_workspace_size(uint64_t n);
/* A workspace of at least spec_encode_nested_workspace_size_items(n, nitems) bytes also keeps the
 * size pass's per-item prefixes for the write pass (faster; same bytes). */
size_t spec_encode_nested_workspace_size_items(uint64_t n, uint64_t nitems);
int spec_encode_nested(const spec_nested_schema *schema, const void *const *outer_columns,
                       const uint8_t *const *outer_heaps, const uint64_t *outer_heap_lens, const uint32_t *item_begin,
                       const void *const *item_columns, const uint8_t *const *item_heaps,
                       const uint64_t *item_heap_lens, uint64_t nitems, uint64_t n, uint8_t *out, uint64_t out_cap,
                       uint64_t *ends, void *workspace, size_t workspace_size, uint64_t *total, void *stream);
/* spec_encode_nested_jit_compile: diagnostic — the hiprtc compile (no GPU needed) of the
 * schema-specialised nested encode kernels; code-object size, 0 if neither schema has one. */
long long spec_encode_nested_jit_compile(const spec_nested_schema *schema);

#ifdef __cplusplus
}
#endif

#endif

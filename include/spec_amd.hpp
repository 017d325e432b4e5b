// spec_amd.hpp — C++17 host API over the C ABI (include/spec_amd.h), header only.
//
// The reference's API is Go (package spec); its toolchain is absent from this image, so the
// compiled host side is this C++ mirror of the reference's batch-relevant surface, named
// after it:
//   spec::OpenMessageBatch      ~ spec.OpenMessageErr + the generated getters, per record
//                                 (msg.go:25-27, internal/types/msg.go:219-475)
//   spec::MessageBatchWriter    ~ spec.NewMessageWriterBuffer + w.Field(tag).<Kind>(v) + w.Build()
//                                 (writer_msg.go:26-31, internal/writer/msg.go:56-60, 99-211)
//   spec::ParseMessageBatch     ~ spec.ParseMessage (msg.go:29-32)
// Errors: a failed call throws spec::Error carrying the spec_rc and its text; per-record
// errors are the status column (the error class OpenMessageErr/ParseMessage would return).
// Buffers are RAII wrappers of spec_device_alloc / spec_host_alloc; nothing here touches a
// record on the CPU.
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "spec_amd.h"

namespace spec {

enum class Kind : uint8_t {
    Bool = SPEC_KIND_BOOL, Byte = SPEC_KIND_BYTE, Int16 = SPEC_KIND_INT16, Int32 = SPEC_KIND_INT32,
    Int64 = SPEC_KIND_INT64, Uint16 = SPEC_KIND_UINT16, Uint32 = SPEC_KIND_UINT32, Uint64 = SPEC_KIND_UINT64,
    Float32 = SPEC_KIND_FLOAT32, Float64 = SPEC_KIND_FLOAT64, Bin64 = SPEC_KIND_BIN64, Bin128 = SPEC_KIND_BIN128,
    Bin256 = SPEC_KIND_BIN256, String = SPEC_KIND_STRING, Bytes = SPEC_KIND_BYTES, List = SPEC_KIND_LIST,
};

inline int Width(Kind k) { return spec_kind_width((int)k); }

struct Error : std::runtime_error {
    int rc;
    Error(int code, const std::string &what)
        : std::runtime_error(what + ": " + spec_strerror(code) + " (hip " + std::to_string(spec_last_hip_error()) + ")"),
          rc(code) {}
};

inline void Check(int rc, const char *what) {
    if (rc != SPEC_OK) throw Error(rc, what);
}

class Stream {
  public:
    Stream() { Check(spec_stream_create(&s_), "spec_stream_create"); }
    ~Stream() {
        if (s_) spec_stream_destroy(s_);
    }
    Stream(const Stream &) = delete;
    Stream &operator=(const Stream &) = delete;
    void Sync() { Check(spec_stream_sync(s_), "spec_stream_sync"); }
    void *get() const { return s_; }

  private:
    void *s_ = nullptr;
};

// Device memory (HBM).
class DeviceBuffer {
  public:
    DeviceBuffer() = default;
    explicit DeviceBuffer(size_t bytes) : n_(bytes) { Check(spec_device_alloc(bytes, &p_), "spec_device_alloc"); }
    ~DeviceBuffer() { reset(); }
    DeviceBuffer(DeviceBuffer &&o) noexcept : p_(std::exchange(o.p_, nullptr)), n_(std::exchange(o.n_, 0)) {}
    DeviceBuffer &operator=(DeviceBuffer &&o) noexcept {
        if (this != &o) {
            reset();
            p_ = std::exchange(o.p_, nullptr);
            n_ = std::exchange(o.n_, 0);
        }
        return *this;
    }
    DeviceBuffer(const DeviceBuffer &) = delete;
    DeviceBuffer &operator=(const DeviceBuffer &) = delete;

    void *data() const { return p_; }
    size_t size() const { return n_; }
    void CopyFrom(const void *host, size_t bytes, Stream &s) { Check(spec_copy_h2d(p_, host, bytes, s.get()), "spec_copy_h2d"); }
    void CopyTo(void *host, size_t bytes, Stream &s) const { Check(spec_copy_d2h(host, p_, bytes, s.get()), "spec_copy_d2h"); }
    template <class T>
    static DeviceBuffer From(const std::vector<T> &v, Stream &s) {
        DeviceBuffer b(v.size() * sizeof(T));
        if (!v.empty()) b.CopyFrom(v.data(), v.size() * sizeof(T), s);
        return b;
    }
    template <class T>
    std::vector<T> ToHost(Stream &s) const {
        std::vector<T> v(n_ / sizeof(T));
        if (!v.empty()) CopyTo(v.data(), v.size() * sizeof(T), s);
        s.Sync();
        return v;
    }

  private:
    void reset() {
        if (p_) spec_device_free(p_);
        p_ = nullptr;
        n_ = 0;
    }
    void *p_ = nullptr;
    size_t n_ = 0;
};

// The fields a generated Write() emits, in write order (internal/lang/generator/message.go:319-439).
class Schema {
  public:
    Schema &Field(uint16_t tag, Kind kind) {
        if (fields_.size() >= SPEC_MAX_FIELDS) throw Error(SPEC_E_INVALID_ARGUMENT, "Schema::Field");
        fields_.push_back({tag, kind});
        return *this;
    }
    size_t Len() const { return fields_.size(); }
    uint16_t Tag(size_t f) const { return fields_[f].first; }
    Kind KindOf(size_t f) const { return fields_[f].second; }
    spec_schema C() const {
        spec_schema s;
        std::memset(&s, 0, sizeof(s));
        s.nfields = (uint32_t)fields_.size();
        for (size_t f = 0; f < fields_.size(); f++) {
            s.fields[f].tag = fields_[f].first;
            s.fields[f].kind = (uint8_t)fields_[f].second;
        }
        return s;
    }

  private:
    std::vector<std::pair<uint16_t, Kind>> fields_;
};

// A batch of encoded records in HBM: stream = records back to back, ends[i] = end of record i.
struct Batch {
    DeviceBuffer stream, ends;
    uint64_t len = 0, n = 0;
};

// Decoded columns of a batch (one per schema field) + the per-record status.
class MessageBatch {
  public:
    const DeviceBuffer &Column(size_t f) const { return cols_[f]; }
    const DeviceBuffer &Status() const { return status_; }
    uint64_t Len() const { return n_; }
    template <class T>
    std::vector<T> Get(size_t f, Stream &s) const { return cols_[f].ToHost<T>(s); }

  private:
    friend MessageBatch OpenMessageBatch(const Schema &, const Batch &, Stream &);
    std::vector<DeviceBuffer> cols_;
    DeviceBuffer status_;
    uint64_t n_ = 0;
};

// For every record: m, err := spec.OpenMessageErr(b); status = class(err); column_f = m.<Kind_f>(tag_f).
inline MessageBatch OpenMessageBatch(const Schema &schema, const Batch &b, Stream &s) {
    MessageBatch m;
    m.n_ = b.n;
    std::vector<void *> ptrs;
    for (size_t f = 0; f < schema.Len(); f++) {
        m.cols_.emplace_back((size_t)b.n * Width(schema.KindOf(f)) + 1);
        ptrs.push_back(m.cols_.back().data());
    }
    m.status_ = DeviceBuffer(b.n + 1);
    spec_schema c = schema.C();
    Check(spec_decode_flat(&c, (const uint8_t *)b.stream.data(), b.len, (const uint64_t *)b.ends.data(), b.n,
                           ptrs.data(), (uint8_t *)m.status_.data(), s.get()),
          "spec_decode_flat");
    return m;
}

// For every record: spec.ParseMessage(b) (recursive validation); returns the status column.
inline DeviceBuffer ParseMessageBatch(const Batch &b, Stream &s, uint32_t head = 0) {
    DeviceBuffer st(b.n + 1);
    Check(spec_parse_messages((const uint8_t *)b.stream.data(), b.len, (const uint64_t *)b.ends.data(), b.n, head,
                              (uint8_t *)st.data(), nullptr, s.get()),
          "spec_parse_messages");
    return st;
}

// For every record: w := NewMessageWriterBuffer(buf); w.Field(tag_f).<Kind_f>(column_f[i])...; w.Build().
class MessageBatchWriter {
  public:
    MessageBatchWriter(const Schema &schema, uint64_t n)
        : schema_(schema), n_(n), cols_(schema.Len(), nullptr), heaps_(schema.Len(), nullptr), lens_(schema.Len(), 0) {}

    // column f: n elements of the kind's width (string/bytes: {u32 off, u32 len} into heap)
    MessageBatchWriter &Field(size_t f, const DeviceBuffer &column, const DeviceBuffer *heap = nullptr) {
        cols_.at(f) = column.data();
        if (heap) {
            heaps_[f] = (const uint8_t *)heap->data();
            lens_[f] = heap->size();
        }
        return *this;
    }

    // Sizes, then (after one host sync for the total) the bytes.
    Batch Build(Stream &s) {
        spec_schema c = schema_.C();
        const size_t ws = spec_encode_flat_workspace_size(n_);
        DeviceBuffer work(ws), total(8);
        Check(spec_encode_flat_size(&c, cols_.data(), n_, work.data(), ws, (uint64_t *)total.data(), s.get()),
              "spec_encode_flat_size");
        uint64_t t = 0;
        total.CopyTo(&t, 8, s);
        s.Sync();
        if (t == ~0ull) throw Error(SPEC_E_INVALID_ARGUMENT, "MessageBatchWriter::Build (encoder error)");
        Batch b;
        b.stream = DeviceBuffer(t ? t : 1);
        b.ends = DeviceBuffer(n_ * 8 + 8);
        b.len = t;
        b.n = n_;
        Check(spec_encode_flat(&c, cols_.data(), heaps_.data(), lens_.data(), n_, (uint8_t *)b.stream.data(), t,
                               (uint64_t *)b.ends.data(), work.data(), ws, (uint64_t *)total.data(), s.get()),
              "spec_encode_flat");
        uint64_t t2 = 0;
        total.CopyTo(&t2, 8, s);
        s.Sync();
        if (t2 != t) throw Error(SPEC_E_INVALID_ARGUMENT, "MessageBatchWriter::Build (span outside its heap)");
        return b;
    }

  private:
    Schema schema_;
    uint64_t n_;
    std::vector<const void *> cols_;
    std::vector<const uint8_t *> heaps_;
    std::vector<uint64_t> lens_;
};

// Pinned host memory (hipHostMalloc): what an mpx connection reads frames into.
class PinnedBuffer {
  public:
    explicit PinnedBuffer(size_t bytes) : n_(bytes) { Check(spec_host_alloc(bytes ? bytes : 1, &p_), "spec_host_alloc"); }
    ~PinnedBuffer() {
        if (p_) spec_host_free(p_);
    }
    PinnedBuffer(const PinnedBuffer &) = delete;
    PinnedBuffer &operator=(const PinnedBuffer &) = delete;
    uint8_t *data() const { return (uint8_t *)p_; }
    size_t size() const { return n_; }

  private:
    void *p_ = nullptr;
    size_t n_ = 0;
};

// The receive side of an mpx connection, batched: records (stream + ends) in pinned host memory
// in, decoded columns + status in pinned host memory out, H2D / decode / D2H overlapped in
// chunks (spec_host_decoder_*).  Outputs are chunk-major: Chunk(k) locates chunk k's columns.
class HostMessageReader {
  public:
    HostMessageReader(const Schema &schema, uint64_t max_records, uint64_t max_bytes, uint32_t chunks = 8)
        : schema_(schema), chunks_(chunks) {
        spec_schema c = schema.C();
        Check(spec_host_decoder_create(&c, max_records, max_bytes, chunks, &d_), "spec_host_decoder_create");
    }
    ~HostMessageReader() { spec_host_decoder_destroy(d_); }
    HostMessageReader(const HostMessageReader &) = delete;
    HostMessageReader &operator=(const HostMessageReader &) = delete;

    uint64_t OutBytes(uint64_t n) const { return spec_host_decoder_out_bytes(d_, n); }
    // For every record i of stream[ends[i-1], ends[i]): OpenMessageErr + the getters (synchronous).
    void Read(const PinnedBuffer &stream, uint64_t stream_len, const PinnedBuffer &ends, uint64_t n,
              PinnedBuffer &out) {
        if (out.size() < OutBytes(n) || ends.size() < n * 8) throw Error(SPEC_E_CAPACITY, "HostMessageReader::Read");
        Check(spec_host_decoder_run(d_, stream.data(), stream_len, (const uint64_t *)ends.data(), n, out.data()),
              "spec_host_decoder_run");
    }
    struct ChunkView {
        uint64_t r0, r1;
        std::vector<uint64_t> col_off; // byte offset of column f of records [r0, r1) in `out`
        uint64_t status_off;
    };
    ChunkView Chunk(uint64_t n, uint32_t k) const {
        ChunkView v;
        v.col_off.resize(schema_.Len() ? schema_.Len() : 1);
        Check(spec_host_decoder_chunk(d_, n, k, &v.r0, &v.r1, v.col_off.data(), &v.status_off),
              "spec_host_decoder_chunk");
        return v;
    }
    uint32_t Chunks() const { return chunks_; }

  private:
    Schema schema_;
    uint32_t chunks_;
    spec_host_decoder *d_ = nullptr;
};

} // namespace spec

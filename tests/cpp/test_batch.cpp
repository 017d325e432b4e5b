// test_batch.cpp — the C++ host API (include/spec_amd.hpp) on the GPU, written the way the
// reference's Go tests are (internal/decode/*_test.go, internal/writer/*_test.go): each case
// builds records, runs the batch call, and checks against the CPU oracle (test infrastructure).
// Built and run by tests/test_gpu_cpp.py.  Exit 0 = all pass.
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "spec_amd.hpp"
#include "spec_oracle.h"

namespace {

std::vector<std::pair<std::string, std::function<void()>>> &registry() {
    static std::vector<std::pair<std::string, std::function<void()>>> r;
    return r;
}
struct Reg {
    Reg(const char *name, std::function<void()> fn) { registry().push_back({name, fn}); }
};
#define TEST(name) \
    void name();   \
    Reg reg_##name(#name, name); \
    void name()
#define REQUIRE(cond)                                                                     \
    do {                                                                                  \
        if (!(cond)) throw std::runtime_error(std::string(__FILE__ ":") + std::to_string(__LINE__) + ": " #cond); \
    } while (0)

const uint16_t kTags[5] = {1, 2, 5, 9, 12};
const uint8_t kKinds[5] = {SPEC_KIND_INT64, SPEC_KIND_STRING, SPEC_KIND_FLOAT64, SPEC_KIND_BOOL, SPEC_KIND_UINT32};

spec::Schema test_schema() {
    spec::Schema s;
    for (int f = 0; f < 5; f++) s.Field(kTags[f], (spec::Kind)kKinds[f]);
    return s;
}

struct HostRecords {
    uint64_t n;
    std::vector<int64_t> i64;
    std::vector<uint32_t> str; // {off, len}
    std::vector<double> f64;
    std::vector<uint8_t> b;
    std::vector<uint32_t> u32;
    std::vector<uint8_t> heap;
    std::vector<uint8_t> stream;
    std::vector<uint64_t> ends;
};

HostRecords test_records(uint64_t n) {
    HostRecords h;
    h.n = n;
    uint64_t x = 42;
    for (uint64_t i = 0; i < n; i++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        h.i64.push_back((int64_t)x >> (x & 63));
        uint32_t len = (uint32_t)(x >> 58);
        h.str.push_back((uint32_t)h.heap.size());
        h.str.push_back(len);
        for (uint32_t k = 0; k < len; k++) h.heap.push_back((uint8_t)('a' + (x >> k) % 26));
        h.f64.push_back((double)(int64_t)x * 1e-3);
        h.b.push_back((x >> 9) & 1);
        h.u32.push_back((uint32_t)(x >> 17));
    }
    const void *cols[5] = {h.i64.data(), h.str.data(), h.f64.data(), h.b.data(), h.u32.data()};
    const uint8_t *heaps[5] = {nullptr, h.heap.data(), nullptr, nullptr, nullptr};
    h.stream.resize(n * 128 + h.heap.size() + 16);
    h.ends.resize(n);
    if (so_encode_flat_batch(5, kTags, kKinds, cols, heaps, n, h.stream.data(), h.stream.size(), h.ends.data()))
        throw std::runtime_error("oracle encode");
    h.stream.resize(n ? h.ends[n - 1] : 0);
    return h;
}

spec::Batch upload(const std::vector<uint8_t> &stream, const std::vector<uint64_t> &ends, spec::Stream &s) {
    spec::Batch b;
    b.stream = spec::DeviceBuffer::From(stream.empty() ? std::vector<uint8_t>(1) : stream, s);
    b.ends = spec::DeviceBuffer::From(ends.empty() ? std::vector<uint64_t>(1) : ends, s);
    b.len = stream.size();
    b.n = ends.size();
    return b;
}

void expect_like_oracle(const spec::MessageBatch &m, const std::vector<uint8_t> &stream,
                        const std::vector<uint64_t> &ends, spec::Stream &s) {
    const uint64_t n = ends.size();
    std::vector<std::vector<uint8_t>> want(5);
    std::vector<void *> wp;
    for (int f = 0; f < 5; f++) {
        want[f].resize(n * spec_kind_width(kKinds[f]) + 1);
        wp.push_back(want[f].data());
    }
    std::vector<uint8_t> wst(n + 1);
    so_decode_flat_batch(5, kTags, kKinds, stream.data(), ends.data(), n, wp.data(), wst.data(), 1);
    auto gst = m.Status().ToHost<uint8_t>(s);
    REQUIRE(std::memcmp(gst.data(), wst.data(), n) == 0);
    for (int f = 0; f < 5; f++) {
        auto g = m.Get<uint8_t>(f, s);
        REQUIRE(std::memcmp(g.data(), want[f].data(), n * spec_kind_width(kKinds[f])) == 0);
    }
}

// internal/bench/parse_test.go:48-111 pattern, as a batch
TEST(TestOpenMessageBatch__should_decode_written_records) {
    spec::Stream s;
    HostRecords h = test_records(5003);
    spec::Batch b = upload(h.stream, h.ends, s);
    spec::MessageBatch m = spec::OpenMessageBatch(test_schema(), b, s);
    expect_like_oracle(m, h.stream, h.ends, s);
    auto st = m.Status().ToHost<uint8_t>(s);
    for (uint64_t i = 0; i < h.n; i++) REQUIRE(st[i] == SPEC_STATUS_OK);
    auto v = m.Get<int64_t>(0, s);
    for (uint64_t i = 0; i < h.n; i++) REQUIRE(v[i] == h.i64[i]);
}

// the mpx receive loop batched: pinned host in, pinned host out (chunk-major), results as above
TEST(TestHostMessageReader__should_decode_host_records) {
    HostRecords h = test_records(20011);
    const uint64_t n = h.n;
    spec::PinnedBuffer stream(h.stream.size()), ends(n * 8);
    std::memcpy(stream.data(), h.stream.data(), h.stream.size());
    std::memcpy(ends.data(), h.ends.data(), n * 8);
    spec::HostMessageReader reader(test_schema(), n, h.stream.size(), 6);
    spec::PinnedBuffer out(reader.OutBytes(n));
    reader.Read(stream, h.stream.size(), ends, n, out);
    std::vector<std::vector<uint8_t>> want(5);
    std::vector<void *> wp;
    for (int f = 0; f < 5; f++) {
        want[f].resize(n * spec_kind_width(kKinds[f]) + 1);
        wp.push_back(want[f].data());
    }
    std::vector<uint8_t> wst(n + 1);
    so_decode_flat_batch(5, kTags, kKinds, h.stream.data(), h.ends.data(), n, wp.data(), wst.data(), 1);
    uint64_t covered = 0;
    for (uint32_t k = 0; k < reader.Chunks(); k++) {
        auto c = reader.Chunk(n, k);
        covered += c.r1 - c.r0;
        REQUIRE(std::memcmp(out.data() + c.status_off, wst.data() + c.r0, c.r1 - c.r0) == 0);
        for (int f = 0; f < 5; f++) {
            const uint64_t w = spec_kind_width(kKinds[f]);
            REQUIRE(std::memcmp(out.data() + c.col_off[f], want[f].data() + c.r0 * w, (c.r1 - c.r0) * w) == 0);
        }
    }
    REQUIRE(covered == n);
}

// internal/decode/msg_test.go:74-143 error classes, as records of one batch
TEST(TestOpenMessageBatch__should_return_error_classes) {
    std::vector<std::vector<uint8_t>> recs = {
        {0x01, 0x46},             // invalid type (a list)
        {0xff, 0x50},             // invalid table size
        {0xff, 0x07, 0xe8, 0x50}, // invalid data size
        {0x00, 0x00, 0x50},       // empty table, empty data: ok
        {},                       // empty: ok
    };
    std::vector<uint8_t> stream;
    std::vector<uint64_t> ends;
    for (auto &r : recs) {
        stream.insert(stream.end(), r.begin(), r.end());
        ends.push_back(stream.size());
    }
    spec::Stream s;
    spec::Batch b = upload(stream, ends, s);
    spec::MessageBatch m = spec::OpenMessageBatch(test_schema(), b, s);
    expect_like_oracle(m, stream, ends, s);
    auto st = m.Status().ToHost<uint8_t>(s);
    REQUIRE(st[0] == SPEC_STATUS_INVALID_TYPE && st[1] == SPEC_STATUS_INVALID_TABLE_SIZE &&
            st[2] == SPEC_STATUS_INVALID_DATA_SIZE && st[3] == SPEC_STATUS_OK && st[4] == SPEC_STATUS_OK);
}

// internal/bench/write_test.go:16-78 pattern, as a batch: bytes identical to the Writer's
TEST(TestMessageBatchWriter__should_write_records_like_writer) {
    spec::Stream s;
    HostRecords h = test_records(7001);
    auto c0 = spec::DeviceBuffer::From(h.i64, s), c1 = spec::DeviceBuffer::From(h.str, s),
         c2 = spec::DeviceBuffer::From(h.f64, s), c3 = spec::DeviceBuffer::From(h.b, s),
         c4 = spec::DeviceBuffer::From(h.u32, s), heap = spec::DeviceBuffer::From(h.heap, s);
    spec::MessageBatchWriter w(test_schema(), h.n);
    w.Field(0, c0).Field(1, c1, &heap).Field(2, c2).Field(3, c3).Field(4, c4);
    spec::Batch b = w.Build(s);
    REQUIRE(b.len == h.stream.size());
    auto out = b.stream.ToHost<uint8_t>(s);
    auto ends = b.ends.ToHost<uint64_t>(s);
    REQUIRE(std::memcmp(out.data(), h.stream.data(), b.len) == 0);
    REQUIRE(std::memcmp(ends.data(), h.ends.data(), h.n * 8) == 0);
}

// internal/types/msg.go:58-82: ParseMessage over the batch
TEST(TestParseMessageBatch__should_validate_records) {
    spec::Stream s;
    HostRecords h = test_records(1000);
    h.stream[h.ends[10] - 1] = 0x63; // record 10: its type byte -> not a message
    spec::Batch b = upload(h.stream, h.ends, s);
    auto st = spec::ParseMessageBatch(b, s).ToHost<uint8_t>(s);
    std::vector<uint8_t> want(h.n);
    std::vector<uint32_t> sizes(h.n);
    so_parse_batch(h.stream.data(), h.ends.data(), h.n, 0, want.data(), sizes.data());
    REQUIRE(std::memcmp(st.data(), want.data(), h.n) == 0);
    REQUIRE(st[10] == SPEC_STATUS_INVALID_TYPE && st[0] == SPEC_STATUS_OK);
}

TEST(TestError__should_carry_rc) {
    spec::Schema bad;
    bad.Field(1, (spec::Kind)42);
    spec::Stream s;
    HostRecords h = test_records(10);
    spec::Batch b = upload(h.stream, h.ends, s);
    bool thrown = false;
    try {
        spec::OpenMessageBatch(bad, b, s);
    } catch (const spec::Error &e) {
        thrown = e.rc == SPEC_E_INVALID_ARGUMENT;
    }
    REQUIRE(thrown);
}

} // namespace

int main() {
    int fails = 0;
    for (auto &t : registry()) {
        try {
            t.second();
            std::printf("PASS %s\n", t.first.c_str());
        } catch (const std::exception &e) {
            fails++;
            std::printf("FAIL %s: %s\n", t.first.c_str(), e.what());
        }
    }
    std::printf("%zu tests, %d failed\n", registry().size(), fails);
    return fails ? 1 : 0;
}

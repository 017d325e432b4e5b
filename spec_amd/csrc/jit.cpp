// jit.cpp — schema-specialised decode and encode kernels, compiled at run time with hiprtc.
//
// The reference decodes through GENERATED code: `spec generate` emits one Go reader per
// schema whose getters call Message.<Kind>(tag) with constant tags
// (internal/lang/generator/message.go:97-186).  This is the MI355X analogue: the first time
// a schema is decoded, decode_core.hpp's kernel body is instantiated for that schema (field
// count, kinds, tags and table order as compile-time constants) and compiled for gfx950
// with hiprtc; the code object is loaded with hipModuleLoadData and cached per (device,
// schema).  The generated kernel keeps the generic path for every record its fast path
// rejects, so results are identical to the precompiled kernel's.
//
// Schemas without a fast path (more than FAST_MAX_FIELDS fields, repeated tags, tags >
// 255) and SPEC_AMD_JIT=0 use the precompiled generic kernel (decode_flat.hip).
//
// Encode: the generated Write() (internal/lang/generator/message.go:319-439) likewise —
// encode_core.hpp's size and write bodies over SpecEnc<schema> (every column load of a
// record issued at once, the table built from registers); any schema of 1..ENC_MAX_FIELDS
// non-list fields.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <dlfcn.h>
#include <sys/stat.h>
#include <utime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "spec_internal.hpp"
#include "tree_core.hpp"

namespace {

// the device sources, embedded at build time (Makefile -> build/rtc_sources.inc)
#include "build/rtc_sources.inc"

struct Entry {
    hipModule_t mod = nullptr;
    hipFunction_t fn[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    bool failed = false;
};

std::mutex g_mu;
std::unordered_map<std::string, Entry> g_cache;
int g_enabled = -1; // -1: read SPEC_AMD_JIT on first use

bool enabled() {
    if (g_enabled < 0) {
        const char *e = getenv("SPEC_AMD_JIT");
        g_enabled = (e && e[0] == '0') ? 0 : 1;
    }
    return g_enabled == 1;
}

bool debug() {
    const char *e = getenv("SPEC_AMD_DEBUG");
    return e && e[0] && e[0] != '0';
}

// Table order a Writer produces (insertion sort, internal/writer/stack_msg.go:37-61).
void writer_order(const spec_schema *s, uint8_t *order, uint16_t *sorted) {
    for (uint32_t f = 0; f < s->nfields; f++) {
        sorted[f] = s->fields[f].tag;
        order[f] = (uint8_t)f;
        for (int i = (int)f; i > 0 && sorted[i - 1] >= sorted[i]; i--) {
            std::swap(sorted[i - 1], sorted[i]);
            std::swap(order[i - 1], order[i]);
        }
    }
}

// The flat decoder's fast path (decode_core.hpp fast_prepare / fast_wide) exists when the
// Writer's table is strictly increasing: any field count, tags <= 255 (small tables) or with a
// tag > 255 (every table big).
bool has_flat_fast_path(const spec_schema *s) {
    if (s->nfields == 0 || s->nfields > SPEC_KFIELDS) return false;
    for (uint32_t f = 0; f < s->nfields; f++)
        if (s->fields[f].kind == SPEC_KIND_LIST) return false;
    uint8_t order[SPEC_KFIELDS];
    uint16_t sorted[SPEC_KFIELDS];
    writer_order(s, order, sorted);
    for (uint32_t k = 0; k < s->nfields; k++) {
        if (sorted[k] == 0) return false;
        if (k && sorted[k] <= sorted[k - 1]) return false;
    }
    return true;
}

// The nested decoder's fast path (register-resident): strictly increasing tags <= 255, at most
// FAST_MAX_FIELDS fields.
bool has_fast_path(const spec_schema *s) {
    if (s->nfields == 0 || s->nfields > (uint32_t)spec::FAST_MAX_FIELDS) return false;
    uint8_t order[SPEC_KFIELDS];
    uint16_t sorted[SPEC_KFIELDS];
    writer_order(s, order, sorted);
    for (uint32_t k = 0; k < s->nfields; k++) {
        if (sorted[k] > 255 || sorted[k] == 0) return false;
        if (k && sorted[k] <= sorted[k - 1]) return false;
    }
    return true;
}

// A schema-specialised encoder exists for 1..ENC_MAX_FIELDS fields without list fields.
constexpr uint32_t ENC_MAX_FIELDS = 32;
bool has_encoder(const spec_schema *s) {
    if (s->nfields == 0 || s->nfields > ENC_MAX_FIELDS) return false;
    for (uint32_t f = 0; f < s->nfields; f++)
        if (s->fields[f].kind == SPEC_KIND_LIST) return false;
    return true;
}

enum Prog { DECODE = 0, ENCODE = 1, NESTED = 2, NESTED_ENC = 3, TREE = 4 };

std::string key_of(const spec_schema *s, int device, Prog p) {
    std::ostringstream k;
    k << (p == ENCODE || p == NESTED_ENC ? "enc:" : "dec:") << device << ':' << (spec::persistent_decode() ? 'p' : 'o') << ':';
    for (uint32_t f = 0; f < s->nfields; f++) k << s->fields[f].tag << '/' << (int)s->fields[f].kind << ',';
    return k.str();
}

// struct <name> { N, kind[], rank[], stag[] }: the fast-path schema of decode_core.hpp
void emit_spec(std::ostringstream &o, const char *name, const spec_schema *s) {
    uint8_t order[SPEC_KFIELDS];
    uint16_t sorted[SPEC_KFIELDS];
    writer_order(s, order, sorted);
    uint8_t rank[SPEC_KFIELDS];
    for (uint32_t k = 0; k < s->nfields; k++) rank[order[k]] = (uint8_t)k;
    o << "struct " << name << " {\n  static constexpr int N = " << s->nfields << ";\n"
      << "  static constexpr uint32_t kind[N] = {";
    for (uint32_t f = 0; f < s->nfields; f++) o << (f ? "," : "") << (int)s->fields[f].kind;
    o << "};\n  static constexpr int rank[N] = {";
    for (uint32_t f = 0; f < s->nfields; f++) o << (f ? "," : "") << (int)rank[f];
    o << "};\n  static constexpr uint32_t stag[N] = {";
    for (uint32_t k = 0; k < s->nfields; k++) o << (k ? "," : "") << sorted[k];
    o << "};\n  static constexpr int order[N] = {";
    for (uint32_t k = 0; k < s->nfields; k++) o << (k ? "," : "") << (int)order[k];
    bool big = false;
    for (uint32_t k = 0; k < s->nfields; k++) big = big || sorted[k] > 255;
    o << "};\n  static constexpr bool big = " << (big ? "true" : "false") << ";\n};\n";
}

// waves per 64-record group of the flat decode (decode_core.hpp decode_flat_pair); build-time A/B
#ifndef SPEC_AB_FLAT_WAVES
#define SPEC_AB_FLAT_WAVES 2
#endif

std::string generate_decode(const spec_schema *s) {
    std::ostringstream o;
    o << "#include \"decode_core.hpp\"\n";
    emit_spec(o, "GenSpec", s);
    const char *pers = spec::persistent_decode() ? "true" : "false";
    // schemas on decode_core.hpp fast_wide get kernels of their own names (traces tell them apart)
    bool big = false;
    for (uint32_t f = 0; f < s->nfields; f++) big = big || s->fields[f].tag > 255;
    const char *w = (s->nfields > (uint32_t)spec::FAST_MAX_FIELDS || big) ? "_wide" : "";
    o << "extern \"C\" __global__ __launch_bounds__(256) void spec_decode_flat" << w << "_jit(spec::DecodeArgs a) {\n"
      << "  spec::decode_flat_entry<" << pers << ", GenSpec>(a);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(256) void spec_decode_flat" << w << "_err_jit(spec::DecodeArgs a) {\n"
      << "  spec::decode_flat_entry<" << pers << ", GenSpec, true>(a);\n}\n";
    // the wave-pair kernel (decode_core.hpp decode_flat_pair), the default launch for every
    // schema (decode_flat.hip SPEC_AB_FLAT_PAIR)
    const int P = SPEC_AB_FLAT_WAVES;
    o << "extern \"C\" __global__ __launch_bounds__(" << 64 * P << ") void spec_decode_flat" << w
      << "_pair_jit(spec::DecodeArgs a) {\n"
      << "  spec::decode_flat_pair<GenSpec, false, " << P << ">(a);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(" << 64 * P << ") void spec_decode_flat" << w
      << "_err_pair_jit(spec::DecodeArgs a) {\n"
      << "  spec::decode_flat_pair<GenSpec, true, " << P << ">(a);\n}\n";
    return o.str();
}

// The nested decode's wave group (decode_nested_core.hpp nested_decode_pair): waves per group
// and item rounds of 64 per wave in flight; build-time A/B only.
#ifndef SPEC_AB_NESTED_WAVES
#define SPEC_AB_NESTED_WAVES 2
#endif
#ifndef SPEC_AB_NESTED_U
#define SPEC_AB_NESTED_U 1
#endif
#ifndef SPEC_AB_NESTED_SELF
#define SPEC_AB_NESTED_SELF 0
#endif

// One-pass nested decode: outer and item fast paths where the schema has one.
std::string generate_nested(const spec_nested_schema *s) {
    std::ostringstream o;
    o << "#include \"decode_nested_core.hpp\"\n";
    const bool fo = has_fast_path(&s->outer), fi = has_fast_path(&s->item);
    if (fo) emit_spec(o, "GenOuter", &s->outer);
    if (fi) emit_spec(o, "GenItem", &s->item);
    const std::string specs = std::string(fo ? "GenOuter" : "spec::RuntimeSpec") + ", " +
                              (fi ? "GenItem" : "spec::RuntimeSpec");
    o << "extern \"C\" __global__ __launch_bounds__(256) void spec_decode_nested_jit(spec::NestedArgs a) {\n"
      << "  spec::nested_decode_body<" << specs << ", true>(a);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(64) void spec_decode_nested2_jit(spec::NestedArgs a) {\n"
      << "  spec::nested_decode_body<" << specs << ", false>(a);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(64) void spec_decode_nested3_jit(spec::NestedArgs a) {\n"
      << "  spec::nested_decode_body<" << specs << ", false, true>(a);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(" << 64 * SPEC_AB_NESTED_WAVES
      << ") void spec_decode_nested_pair_jit(spec::NestedArgs a) {\n"
      << "  spec::nested_decode_pair<" << specs << ", " << SPEC_AB_NESTED_U << ", " << SPEC_AB_NESTED_WAVES
      << ", " << (SPEC_AB_NESTED_SELF ? "true" : "false") << ">(a);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(" << 64 * SPEC_AB_NESTED_WAVES
      << ") void spec_decode_nested_pairlb_jit(spec::NestedArgs a) {\n"
      << "  spec::nested_decode_pair<" << specs << ", " << SPEC_AB_NESTED_U << ", " << SPEC_AB_NESTED_WAVES
      << ", false, true>(a);\n}\n";
    return o.str();
}

// The generated Write() of internal/lang/generator/message.go:319-439 as constants: fields in
// write order, the Writer's table order, IsBigMessage forced by a tag > 255.
void emit_enc_spec(std::ostringstream &o, const char *name, const spec_schema *s) {
    uint8_t order[SPEC_KFIELDS];
    uint16_t sorted[SPEC_KFIELDS];
    writer_order(s, order, sorted);
    bool big = false;
    o << "struct " << name << " {\n  static constexpr int N = " << s->nfields << ";\n"
      << "  static constexpr uint32_t kind[N] = {";
    for (uint32_t f = 0; f < s->nfields; f++) o << (f ? "," : "") << (int)s->fields[f].kind;
    o << "};\n  static constexpr uint32_t tag[N] = {";
    for (uint32_t f = 0; f < s->nfields; f++) {
        o << (f ? "," : "") << s->fields[f].tag;
        big |= s->fields[f].tag > 255;
    }
    o << "};\n  static constexpr int order[N] = {";
    for (uint32_t k = 0; k < s->nfields; k++) o << (k ? "," : "") << (int)order[k];
    o << "};\n  static constexpr bool big_forced = " << (big ? "true" : "false") << ";\n};\n";
}

// Nested encode: SpecEnc for the outer schema (its list field handled by the nested encoder's
// hooks) and for the item schema, RuntimeEnc for a side without a specialised encoder.
bool has_outer_encoder(const spec_schema *s) { return s->nfields > 0 && s->nfields <= ENC_MAX_FIELDS; }
bool nested_wide(const spec_nested_schema *s);
bool has_nested_encoder(const spec_nested_schema *s) {
    return !nested_wide(s) && (has_outer_encoder(&s->outer) || has_encoder(&s->item));
}

// build-time A/B of the nested pair write pass (encode_nested_core.hpp), passed into the
// generated source: the JIT compile sees only what the source defines
#ifndef SPEC_AB_NENC_SPLIT
#define SPEC_AB_NENC_SPLIT 45
#endif
#ifndef SPEC_AB_NENC_SKIP
#define SPEC_AB_NENC_SKIP 0
#endif
std::string generate_nested_encode(const spec_nested_schema *s) {
    std::ostringstream o;
    if (SPEC_AB_NENC_SPLIT != 45) o << "#define SPEC_AB_NENC_SPLIT " << SPEC_AB_NENC_SPLIT << "\n";
    if (SPEC_AB_NENC_SKIP) o << "#define SPEC_AB_NENC_SKIP " << SPEC_AB_NENC_SKIP << "\n";
    o << "#include \"encode_nested_core.hpp\"\n";
    const bool fo = has_outer_encoder(&s->outer), fi = has_encoder(&s->item);
    if (fo) emit_enc_spec(o, "GenOuter", &s->outer);
    if (fi) emit_enc_spec(o, "GenItem", &s->item);
    o << "using OP = " << (fo ? "spec::SpecEnc<GenOuter>" : "spec::RuntimeEnc") << ";\n"
      << "using IP = " << (fi ? "spec::SpecEnc<GenItem>" : "spec::RuntimeEnc") << ";\n"
      << "extern \"C\" __global__ __launch_bounds__(256) void spec_encode_nested_size_jit(spec::NestedEncodeArgs a) {\n"
      << "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
      << "  spec::nested_enc_size_body<OP, IP>(a, smem);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(256) void spec_encode_nested_write_jit(spec::NestedEncodeArgs a) {\n"
      << "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
      << "  spec::nested_enc_write_body<OP, IP>(a, smem);\n}\n";
    if (fo) // the write pass on wave pairs (needs the outer list field at a constant index)
        o << "extern \"C\" __global__ __launch_bounds__(512) void spec_encode_nested_write_pair_jit(spec::NestedEncodeArgs a) {\n"
          << "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
          << "  spec::nested_enc_write_pair_body<OP, IP>(a, smem);\n}\n";
    return o.str();
}

// The write pass on wave pairs (encode_core.hpp encode_write_pair_body): wave 0 takes fields
// [0, H), wave 1 fields [H, N) plus the table and trailer.  H balances a per-kind emission cost
// (instructions of the HEAD_ST4 emitter: a string's heap copy and funnel shifts dominate, the
// table + trailer costs about two strings' worth for 16 fields); 0 = no pair kernel (one field).
// Build-time A/B (round 6): bit-exact (204 flat/wide/golden/C-ABI GPU tests), but Flat16 encode
// 0.1255-0.1293 ms with pairs vs 0.1249-0.1287 without (gpurun_out/encab1, three alternating runs
// on one box): a one-wave group already has all 64 records' loads in flight, so a second wave per
// slab adds issue slots, not memory parallelism.  Off by default.
#ifndef SPEC_AB_ENC_PAIR
#define SPEC_AB_ENC_PAIR 0
#endif
int enc_pair_split(const spec_schema *s) {
    const int n = (int)s->nfields;
    if (!SPEC_AB_ENC_PAIR || n < 2) return 0;
    auto cost = [](int k) {
        switch (k) {
        case SPEC_KIND_BOOL: case SPEC_KIND_BYTE: return 8;
        case SPEC_KIND_FLOAT32: return 10;
        case SPEC_KIND_INT64: case SPEC_KIND_UINT64: return 14;
        case SPEC_KIND_BIN128: return 16;
        case SPEC_KIND_BIN256: return 28;
        case SPEC_KIND_STRING: case SPEC_KIND_BYTES: return 100;
        }
        return 12; // 16/32-bit ints, float64, bin64
    };
    int total = 40 + 5 * n, pre[SPEC_KFIELDS + 1] = {0};
    for (int f = 0; f < n; f++) {
        pre[f + 1] = pre[f] + cost(s->fields[f].kind);
        total += cost(s->fields[f].kind);
    }
    int best = 1, best_max = 1 << 30;
    for (int h = 1; h < n; h++) {
        const int m = std::max(pre[h], total - pre[h]);
        if (m < best_max) {
            best_max = m;
            best = h;
        }
    }
    return best;
}

std::string generate_encode(const spec_schema *s) {
    std::ostringstream o;
    o << "#include \"encode_core.hpp\"\n";
    emit_enc_spec(o, "GenEnc", s);
    o << "using P = spec::SpecEnc<GenEnc>;\n"
      << "extern \"C\" __global__ __launch_bounds__(256) void spec_encode_size_jit(spec::EncodeArgs a) {\n"
      << "  spec::encode_size_body<P>(a);\n}\n"
      << "extern \"C\" __global__ __launch_bounds__(256) void spec_encode_write_jit(spec::EncodeArgs a) {\n"
      << "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
      << "  spec::encode_write_body<P>(a, smem);\n}\n";
    if (const int h = enc_pair_split(s))
        o << "extern \"C\" __global__ __launch_bounds__(512) void spec_encode_write_pair_jit(spec::EncodeArgs a) {\n"
          << "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
          << "  spec::encode_write_pair_body<P, " << h << ">(a, smem);\n}\n";
    return o.str();
}

const char *prog_name(Prog p) {
    return p == ENCODE       ? "spec_encode_jit.hip"
           : p == TREE       ? "spec_tree_jit.hip"
           : p == NESTED     ? "spec_decode_nested_jit.hip"
           : p == NESTED_ENC ? "spec_encode_nested_jit.hip"
                             : "spec_decode_flat_jit.hip";
}

// hiprtc compile only; returns the code object (empty on failure)
std::vector<char> compile_uncached(const std::string &src, Prog p, const char *const *opts_in, int nopts) {
    const char *hdr_src[7] = {kSpecDeviceHpp, kDecodeCoreHpp, kEncodeCoreHpp, kDecodeNestedCoreHpp,
                              kEncodeNestedCoreHpp, kTreeCoreHpp, kTreeDecodeCoreHpp};
    const char *hdr_name[7] = {"spec_device.hpp", "decode_core.hpp", "encode_core.hpp", "decode_nested_core.hpp",
                               "encode_nested_core.hpp", "tree_core.hpp", "tree_decode_core.hpp"};
    // SPEC_AMD_JIT_DUMP=prefix: the source is written before the compile (a slow compile can be
    // inspected while it runs), the code object after it
    if (const char *d = getenv("SPEC_AMD_JIT_DUMP")) {
        const std::string base = std::string(d) + (p == ENCODE       ? "encode"
                                                   : p == TREE       ? "tree"
                                                   : p == NESTED     ? "nested"
                                                   : p == NESTED_ENC ? "nested_encode"
                                                                     : "decode");
        if (FILE *f = fopen((base + ".hip").c_str(), "w")) {
            fwrite(src.data(), 1, src.size(), f);
            fclose(f);
        }
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), prog_name(p), 7, hdr_src, hdr_name) != HIPRTC_SUCCESS) return {};
    // the product kernels are compiled with fixed options only: no environment variable can
    // change what a kernel computes
    std::vector<const char *> opts(opts_in, opts_in + nopts);
    hiprtcResult rc = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
    if (rc != HIPRTC_SUCCESS || debug()) {
        size_t ls = 0;
        hiprtcGetProgramLogSize(prog, &ls);
        if (ls > 1) {
            std::vector<char> log(ls + 1, 0);
            hiprtcGetProgramLog(prog, log.data());
            fprintf(stderr, "spec_amd jit: %s\n", log.data());
        }
    }
    if (rc != HIPRTC_SUCCESS) {
        fprintf(stderr, "spec_amd jit: hiprtc compile of %s failed; the generic kernel is used\n", prog_name(p));
        hiprtcDestroyProgram(&prog);
        return {};
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    std::vector<char> code(cs);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    if (const char *d = getenv("SPEC_AMD_JIT_DUMP")) { // the code object (ISA inspection)
        std::string base = std::string(d) + (p == ENCODE       ? "encode"
                                             : p == TREE       ? "tree"
                                             : p == NESTED     ? "nested"
                                             : p == NESTED_ENC ? "nested_encode"
                                                               : "decode");
        if (FILE *f = fopen((base + ".co").c_str(), "wb")) {
            fwrite(code.data(), 1, code.size(), f);
            fclose(f);
        }
    }
    return code;
}

// ---- on-disk code-object cache -----------------------------------------------------------
// A compile costs ~3 s per (schema, kernel set); its result depends only on the generated
// source, the embedded headers and the options, so it is cached under <libdir>/jit_cache
// (next to libspec_amd.so: build() fills it for the benchmark schemas, and it travels with the
// library) or, where that is not writable, $XDG_CACHE_HOME/spec_amd or ~/.cache/spec_amd.
uint64_t fnv1a(uint64_t h, const char *p, size_t n) {
    for (size_t i = 0; i < n; i++) h = (h ^ (uint8_t)p[i]) * 0x100000001b3ull;
    return h;
}

std::string lib_dir() {
    Dl_info info;
    if (dladdr((void *)&fnv1a, &info) && info.dli_fname) {
        std::string f = info.dli_fname;
        size_t k = f.rfind('/');
        return k == std::string::npos ? std::string(".") : f.substr(0, k);
    }
    return ".";
}

std::vector<std::string> cache_dirs() {
    std::vector<std::string> v = {lib_dir() + "/jit_cache"};
    if (const char *x = getenv("XDG_CACHE_HOME")) v.push_back(std::string(x) + "/spec_amd");
    else if (const char *h = getenv("HOME")) v.push_back(std::string(h) + "/.cache/spec_amd");
    return v;
}

bool read_file(const std::string &path, std::vector<char> &out) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    bool ok = n > 0 && fread(out.data(), 1, (size_t)n, f) == (size_t)n;
    fclose(f);
    return ok;
}

void write_cache(const std::string &name, const std::vector<char> &code) {
    for (const std::string &d : cache_dirs()) {
        mkdir(d.c_str(), 0755); // best effort; a missing parent makes the open below fail
        static std::atomic<unsigned> seq{0}; // concurrent compiles (threads) of one process
        const std::string tmp = d + "/." + name + "." + std::to_string(getpid()) + "." + std::to_string(seq++);
        FILE *f = fopen(tmp.c_str(), "wb");
        if (!f) continue;
        bool ok = fwrite(code.data(), 1, code.size(), f) == code.size();
        ok = (fclose(f) == 0) && ok;
        if (ok && rename(tmp.c_str(), (d + "/" + name).c_str()) == 0) return;
        unlink(tmp.c_str());
    }
}

std::vector<char> compile_source(const std::string &src, Prog p) {
    static const char *const kOpts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    uint64_t h = 0xcbf29ce484222325ull;
    h = fnv1a(h, src.data(), src.size());
    for (const char *hs : {kSpecDeviceHpp, kDecodeCoreHpp, kEncodeCoreHpp, kDecodeNestedCoreHpp, kEncodeNestedCoreHpp,
                           kTreeCoreHpp, kTreeDecodeCoreHpp})
        h = fnv1a(h, hs, strlen(hs) + 1);
    for (const char *o : kOpts) h = fnv1a(h, o, strlen(o) + 1);
    char name[64];
    snprintf(name, sizeof name, "%016llx.co", (unsigned long long)h);
    std::vector<char> cached;
    const bool dump = getenv("SPEC_AMD_JIT_DUMP") != nullptr; // diagnostic: always compile (and dump)
    for (const std::string &d : cache_dirs())
        if (!dump && read_file(d + "/" + name, cached)) {
            utime((d + "/" + name).c_str(), nullptr); // in use: build() prunes entries it did not touch
            return cached;
        }
    std::vector<char> code = compile_uncached(src, p, kOpts, (int)(sizeof kOpts / sizeof kOpts[0]));
    if (!code.empty()) write_cache(name, code);
    return code;
}

std::vector<char> compile_code(const spec_schema *s, Prog p) {
    return compile_source(p == ENCODE ? generate_encode(s) : generate_decode(s), p);
}

Entry load(const std::vector<char> &code, Prog p) {
    Entry e;
    if (code.empty()) {
        e.failed = true;
        return e;
    }
    const char *names[4][4] = {{"spec_decode_flat_jit", "spec_decode_flat_err_jit", "spec_decode_flat_pair_jit",
                                "spec_decode_flat_err_pair_jit"},
                               {"spec_encode_size_jit", "spec_encode_write_jit", nullptr, nullptr}, // (+ the pair kernel, optional)
                               {"spec_decode_nested_jit", "spec_decode_nested2_jit", "spec_decode_nested3_jit",
                                "spec_decode_nested_pair_jit"},
                               {"spec_encode_nested_size_jit", "spec_encode_nested_write_jit", nullptr, nullptr}};
    bool ok = hipModuleLoadData(&e.mod, code.data()) == hipSuccess;
    if (ok && p == DECODE && hipModuleGetFunction(&e.fn[0], e.mod, names[p][0]) != hipSuccess) {
        (void)hipGetLastError(); // a wide / big-table schema (generate_decode): its own kernel names
        names[p][0] = "spec_decode_flat_wide_jit";
        names[p][1] = "spec_decode_flat_wide_err_jit";
        names[p][2] = "spec_decode_flat_wide_pair_jit";
        names[p][3] = "spec_decode_flat_wide_err_pair_jit";
    }
    for (int i = 0; ok && i < 4; i++)
        if (names[p][i]) ok = hipModuleGetFunction(&e.fn[i], e.mod, names[p][i]) == hipSuccess;
    if (ok && p == ENCODE && hipModuleGetFunction(&e.fn[2], e.mod, "spec_encode_write_pair_jit") != hipSuccess) {
        (void)hipGetLastError(); // a one-field schema has no pair kernel
        e.fn[2] = nullptr;
    }
    if (ok && p == NESTED && hipModuleGetFunction(&e.fn[4], e.mod, "spec_decode_nested_pairlb_jit") != hipSuccess) {
        (void)hipGetLastError();
        e.fn[4] = nullptr;
    }
    if (ok && p == NESTED_ENC &&
        hipModuleGetFunction(&e.fn[2], e.mod, "spec_encode_nested_write_pair_jit") != hipSuccess) {
        (void)hipGetLastError(); // no specialised outer encoder: no pair kernel
        e.fn[2] = nullptr;
    }
    if (!ok) {
        (void)hipGetLastError();
        e.failed = true;
        for (hipFunction_t &f : e.fn) f = nullptr;
    }
    return e;
}

// cached per key; make() returns the code object. nullptr => use the generic kernel
template <class Make>
const Entry *lookup_key(const std::string &k, Prog p, Make make) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_cache.find(k);
    if (it == g_cache.end()) {
        Entry e = load(make(), p);
        if (e.failed) fprintf(stderr, "spec_amd jit: compile/load failed, generic kernel in use\n");
        it = g_cache.emplace(k, e).first;
    }
    return it->second.failed ? nullptr : &it->second;
}

const Entry *lookup(const spec_schema *s, Prog p) {
    if (!enabled() || s->nfields > SPEC_KFIELDS) return nullptr; // wide schemas: generic kernels
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    // the last few (device, program, schema) answers of this thread: a repeated call (every
    // launch of a steady-state loop, one per device in spec_shard_decode) skips building the key
    // string and the locked map lookup
    struct Hit {
        bool valid = false;
        int dev = 0, prog = 0;
        uint32_t nfields = 0;
        spec_field f[SPEC_KFIELDS];
        const Entry *e = nullptr;
    };
    thread_local Hit hits[8];
    thread_local unsigned next = 0;
    const size_t fb = (size_t)s->nfields * sizeof(spec_field);
    for (const Hit &h : hits)
        if (h.valid && h.dev == dev && h.prog == (int)p && h.nfields == s->nfields && memcmp(h.f, s->fields, fb) == 0)
            return h.e;
    const Entry *e = (p == ENCODE ? has_encoder(s) : has_flat_fast_path(s))
                         ? lookup_key(key_of(s, dev, p), p, [&] { return compile_code(s, p); })
                         : nullptr;
    Hit &h = hits[next++ & 7];
    h.valid = true;
    h.dev = dev;
    h.prog = (int)p;
    h.nfields = s->nfields;
    memcpy(h.f, s->fields, fb);
    h.e = e;
    return e;
}

// a nested kernel is worth compiling when the outer or the item schema has a fast path
// (a half of more than SPEC_KFIELDS fields: the nested schema is decoded in field chunks by the
// run-time kernels, capi.hip nested_decode_chunks, never by a generated kernel)
bool nested_wide(const spec_nested_schema *s) {
    return s->outer.nfields > (uint32_t)SPEC_KFIELDS || s->item.nfields > (uint32_t)SPEC_KFIELDS;
}
bool has_nested_fast_path(const spec_nested_schema *s) {
    return !nested_wide(s) && (has_fast_path(&s->outer) || has_fast_path(&s->item));
}

const Entry *lookup_nested(const spec_nested_schema *s) {
    if (!enabled() || !has_nested_fast_path(s)) return nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    const std::string k = key_of(&s->outer, dev, NESTED) + "|" + key_of(&s->item, dev, NESTED);
    return lookup_key(k, NESTED, [&] { return compile_source(generate_nested(s), NESTED); });
}

const Entry *lookup_nested_encode(const spec_nested_schema *s) {
    if (!enabled() || !has_nested_encoder(s)) return nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    const std::string k = key_of(&s->outer, dev, NESTED_ENC) + "|" + key_of(&s->item, dev, NESTED_ENC) + "|n";
    return lookup_key(k, NESTED_ENC, [&] { return compile_source(generate_nested_encode(s), NESTED_ENC); });
}


// ---- schema trees: the generated readers, one kernel per decode group -------------------------
// For every group root x (the records or a list table) whose message tables qualify (direct
// tags unique and <= 255), a kernel spec_tree_group_<x> whose row code is the generated reader
// of internal/lang/generator/message.go:97-186 with every tag, kind, rank and column index a
// constant: tree_open checks the table against the schema's tag set once, every getter is then
// one table read and a kind-specialised decode; a row whose table does not qualify (unsorted,
// big, foreign tags) runs the run-time reader (tree_message_row), so results never depend on
// which path ran.  Structs are the generated Decode (struct.go:75-113), members last-first.

using spec::TreeDesc;
using spec::TField;
using spec::TTable;

bool tree_table_ok(const TreeDesc &D, uint32_t t) {
    const TTable &T = D.t[t];
    if (T.shape != spec::SHAPE_MESSAGE) return true;
    if (T.nd > 64) return false;
    bool seen[256] = {false};
    for (uint32_t k = 0; k < T.nd; k++) {
        const uint32_t tag = D.f[D.direct[T.d0 + k]].tag;
        if (tag > 255 || seen[tag]) return false;
        seen[tag] = true;
    }
    return true;
}

bool tree_group_ok(const TreeDesc &D, uint32_t x) {
    const TTable &T = D.t[x];
    // a group of more than 24 tables (sub-messages decoded with their owner) runs the run-time
    // kernel: its generated reader is inlined per source and wave variant
    if (T.gn > 24) return false;
    for (uint32_t g = 0; g < T.gn; g++)
        if (!tree_table_ok(D, D.group[T.g0 + g])) return false;
    return true;
}

std::string col_expr(int c) {
    if (c < 0) return "(void *)nullptr";
    return "B.cols[" + std::to_string(c) + "]";
}

// the members of struct field sf, last first, decoded below OFF down to LB (depth d variables)
void gen_struct_members(std::ostringstream &o, const TreeDesc &D, uint32_t sf, const std::string &LB,
                        const std::string &OFF, int d, const std::string &ind) {
    const TField &F = D.f[sf];
    for (int k = (int)F.nmem - 1; k >= 0; k--) {
        const uint32_t mi = D.members[F.mem0 + k];
        const TField &M = D.f[mi];
        if (M.kind == spec::K_STRUCT) {
            const std::string S = "S" + std::to_string(d + 1), Z = "dz" + std::to_string(d + 1),
                              O2 = "off" + std::to_string(d + 1);
            o << ind << "if (" << OFF << " > " << LB << ") { // inner struct, field " << mi << "\n"
              << ind << "  long long " << S << "; uint32_t " << Z << ";\n"
              << ind << "  sst = struct_open(s, " << LB << ", " << OFF << ", " << S << ", " << Z << ");\n"
              << ind << "  if (sst != ST_OK) break;\n"
              << ind << "  long long " << O2 << " = " << S << " + " << Z << ";\n";
            gen_struct_members(o, D, mi, S, O2, d + 1, ind + "  ");
            o << ind << "  " << OFF << " = " << S << ";\n" << ind << "}\n";
        } else {
            o << ind << "{ Val v; int n; const bool ok = decode_value_kn<" << (int)M.kind << ">(s, " << LB << ", " << OFF
              << ", 0, v, n);\n"
              << ind << "  if (" << col_expr(M.col) << ") store_value_k<" << (int)M.kind << ">(" << col_expr(M.col)
              << ", row, v);\n"
              << ind << "  if (!ok) { sst = ST_INVALID_VALUE; break; }\n"
              << ind << "  " << OFF << " -= n; }\n";
        }
    }
}

// sst = the generated Decode of struct field sf over [LO, E) (tree_core.hpp tree_struct)
void gen_struct(std::ostringstream &o, const TreeDesc &D, uint32_t sf, const std::string &LO, const std::string &E,
                const std::string &ind) {
    const TField &F = D.f[sf];
    for (uint32_t i = sf + 1; i < F.send; i++) {
        const TField &M = D.f[i];
        if (M.kind == spec::K_STRUCT || M.col < 0) continue;
        o << ind << "if (" << col_expr(M.col) << ") store_value_k<" << (int)M.kind << ">(" << col_expr(M.col)
          << ", row, Val{0, 0, 0, 0});\n";
    }
    o << ind << "if (" << E << " > " << LO << ") do {\n"
      << ind << "  long long S0; uint32_t dz0;\n"
      << ind << "  sst = struct_open(s, " << LO << ", " << E << ", S0, dz0);\n"
      << ind << "  if (sst != ST_OK) break;\n"
      << ind << "  long long off0 = S0 + dz0;\n";
    gen_struct_members(o, D, sf, "S0", "off0", 0, ind + "  ");
    o << ind << "} while (0);\n";
}

// a message table's row: lo/hi expressions, its status column written (root: a panicked range
// is ST_PANIC)
// sel (the root table of a wave pair, gen_pair_rows): only the direct fields k with sel[k] are
// decoded, and the table's status and *Err bits go to ro (RowOut) for the pair's exchange
void gen_message_table(std::ostringstream &o, const TreeDesc &D, uint32_t t, const std::string &lo,
                       const std::string &hi, bool root, const std::vector<char> *sel = nullptr,
                       const std::string &fallback = "tree_message_fallback", const std::string &on_bad = "") {
    const TTable &T = D.t[t];
    auto skip = [&](uint32_t k) { return sel && !(*sel)[k]; };
    uint64_t m[4] = {0, 0, 0, 0};
    for (uint32_t k = 0; k < T.nd; k++) {
        const uint32_t tag = D.f[D.direct[T.d0 + k]].tag;
        m[tag >> 6] |= 1ull << (tag & 63);
    }
    o << "  { // table " << t << "\n"
      << "    const long long tlo = " << lo << ", thi = " << hi << ";\n"
      << "    const TOpen o = tree_open<" << T.nd << ", 0x" << std::hex << m[0] << "ull, 0x" << m[1] << "ull, 0x" << m[2]
      << "ull, 0x" << m[3] << "ull" << std::dec << ">(s, tlo, thi);\n";
    if (!on_bad.empty()) o << "    if (o.st != ST_OK) { " << on_bad << " } // the owner field's *Err bit\n";
    o << "    uint32_t st;\n"
      << "    if (o.fast) {\n"
      << "      st = o.st;\n"
      << "      const long long ds = o.ds;\n"
      << "      uint64_t *errp = " << (T.err_col >= 0 ? "(uint64_t *)" + col_expr(T.err_col) : std::string("nullptr"))
      << ";\n"
      << "      uint64_t errs = 0;\n";
    // the scalar fields first, as straight-line code (the kernel runs only with every column
    // present): every table read and value window of the table issued before any decode, so
    // the LDS round trips overlap; windows are read for the type a Writer emits, and a field of
    // another accepted type (ints of another width, float32 <-> float64) is decoded again
    // with the general window below
    bool any_nt = false;
    for (uint32_t k = 0; k < T.nd; k++) {
        const TField &F = D.f[D.direct[T.d0 + k]];
        if (F.kind < spec::K_BOOL || F.kind > spec::K_BYTES || skip(k)) continue;
        o << "      const long long end" << k << " = tree_end<" << F.rank << ">(s, o);\n"
          << "      const long long e" << k << " = end" << k << " > 0 ? ds + end" << k << " : ds;\n"
          << "      const Win w" << k << " = load_win<" << (int)F.kind << ", true>(s, e" << k << ");\n";
    }
    o << "      bool slow = false;\n";
    for (uint32_t k = 0; k < T.nd; k++) {
        const TField &F = D.f[D.direct[T.d0 + k]];
        if (F.kind < spec::K_BOOL || F.kind > spec::K_BYTES || skip(k)) continue;
        const uint32_t nt = spec::cross_kind_type(F.kind);
        o << "      bool ok" << k << " = true;\n"
          << "      Val v" << k << " = decode_tail_k<" << (int)F.kind << ", true>(w" << k << ", ds, e" << k << ", 0, &ok" << k
          << ");\n";
        if (nt) {
            any_nt = true;
            o << "      const bool nat" << k << " = end" << k << " <= 0 || ((uint32_t)w" << k << ".t.q0 & 0xff) == " << nt
              << "u;\n"
              << "      slow |= !nat" << k << ";\n";
        }
    }
    if (any_nt) {
        o << "      if (slow) {\n";
        for (uint32_t k = 0; k < T.nd; k++) {
            const TField &F = D.f[D.direct[T.d0 + k]];
            if (F.kind < spec::K_BOOL || F.kind > spec::K_BYTES || !spec::cross_kind_type(F.kind) || skip(k)) continue;
            o << "        if (!nat" << k << ") v" << k << " = decode_tail_k<" << (int)F.kind << ">(load_win<" << (int)F.kind
              << ">(s, e" << k << "), ds, e" << k << ", 0, &ok" << k << ");\n";
        }
        o << "      }\n";
    }
    for (uint32_t k = 0; k < T.nd; k++) {
        const TField &F = D.f[D.direct[T.d0 + k]];
        if (F.kind < spec::K_BOOL || F.kind > spec::K_BYTES || skip(k)) continue;
        const std::string bit = k < 64 ? "(1ull << " + std::to_string(k) + ")" : "0ull";
        o << "      store_value_k<" << (int)F.kind << ">(" << col_expr(F.col) << ", row, v" << k << ");\n"
          << "      errs |= (ok" << k << " || end" << k << " <= 0) ? 0ull : " << bit << ";\n";
    }
    for (uint32_t k = 0; k < T.nd; k++) {
        const uint32_t fi = D.direct[T.d0 + k];
        const TField &F = D.f[fi];
        if ((F.kind >= spec::K_BOOL && F.kind <= spec::K_BYTES) || skip(k)) continue;
        const std::string bit = k < 64 ? "(1ull << " + std::to_string(k) + ")" : "0ull";
        o << "      { // field " << fi << " tag " << F.tag << " kind " << (int)F.kind << "\n"
          << "        const long long end = tree_end<" << F.rank << ">(s, o);\n";
        switch (F.kind) {
        case spec::K_MESSAGE:
            o << "        const long long e = end >= 0 ? ds + end : ds;\n"
              << "        store_u8(" << col_expr(F.present) << ", row, end >= 0 ? 1u : 0u);\n"
              << "        gr[" << D.t[F.table].gslot << " * 64] = end >= 0 ? make_uint2((uint32_t)ds, (uint32_t)e) : make_uint2(0, 0);\n";
            // (its *Err bit — the sub-message's trailer invalid — is set by the sub-table's own
            // tree_open over the same range, gen_sub_tables: the trailer is parsed once)
            break;
        case spec::K_LIST:
            o << "        const long long e = end >= 0 ? ds + end : ds;\n"
              << "        store_u8(" << col_expr(F.present) << ", row, end >= 0 ? 1u : 0u);\n"
              << "        uint32_t cnt = 0;\n"
              << "        uint4 h = make_uint4(0, 0, 0, 0);\n"
              << "        if (e > ds) {\n"
              << "          const Trailer lt = parse_trailer<true>(s, ds, e);\n"
              << "          if (lt.st == ST_OK) {\n"
              << "            cnt = lt.tsize / (lt.big ? 4u : 2u);\n"
              << "            h = make_uint4((uint32_t)lt.tstart, (uint32_t)lt.dstart, lt.dsize, cnt | (lt.big ? 0x80000000u : 0u));\n"
              << "          } else {\n"
              << "            errs |= " << bit << ";\n"
              << "          }\n"
              << "        }\n"
              << "        B.cnt[" << F.table << "][row] = cnt;\n"
              << "        B.lh[" << F.table << "][row] = h;\n";
            break;
        case spec::K_STRUCT:
            o << "        const long long e = end >= 0 ? ds + end : ds;\n"
              << "        uint32_t sst = ST_OK;\n";
            gen_struct(o, D, fi, "ds", "e", "        ");
            o << "        if (sst == ST_PANIC) st = ST_PANIC;\n"
              << "        if (sst != ST_OK) errs |= " << bit << ";\n";
            break;
        case spec::K_ANY:
            o << "        const long long e = end >= 0 ? ds + end : ds;\n"
              << "        long long n = 0;\n"
              << "        uint2 sp = make_uint2(0, 0);\n"
              << "        if (e > ds) {\n"
              << "          if (type_size_inl(s, ds, e, n)) {\n"
              << "            if (n < 0) st = ST_PANIC;\n"
              << "            else if (n > 0 && n <= e - ds) sp = make_uint2((uint32_t)(e - n), (uint32_t)n);\n"
              << "          } else {\n"
              << "            errs |= " << bit << ";\n"
              << "          }\n"
              << "        }\n"
              << "        if (" << col_expr(F.col) << ") ((uint2 *)" << col_expr(F.col) << ")[row] = sp;\n"
              << "        store_u8(" << col_expr(F.present) << ", row, sp.y ? s.u8((long long)sp.x + sp.y - 1) : 0u);\n";
            break;
        default:
            break;
        }
        o << "      }\n";
    }
    if (sel) {
        o << "      (void)errp;\n      ro.errs = errs;\n"
          << "    } else {\n"
          << "      st = " << fallback << "(s, D, B, " << t << "u, row, tlo, thi, gr);\n"
          << "    }\n"
          << "    ro.st = st;\n    ro.fast = o.fast ? 1u : 0u;\n"
          << "  }\n";
        return;
    }
    o << "      if (errp) errp[row] = errs;\n"
      << "    } else {\n"
      << "      st = " << fallback << "(s, D, B, " << t << "u, row, tlo, thi, gr);\n"
      << "    }\n"
      << "    store_u8(" << col_expr(T.status_col) << ", row, " << (root ? "panic ? (uint32_t)ST_PANIC : st" : "st")
      << ");\n"
      << "  }\n";
}

// an eager writer's table in the Writer's tie-sorted order over the present fields (e<k> marks),
// then its trailer; `data`, `nf`, `big` in scope
void gen_table_trailer(std::ostringstream &o, const TreeDesc &D, const TTable &T) {
    o << "  if (!big) {\n";
    for (uint32_t j = 0; j < T.nd; j++) {
        const uint32_t fi = D.sorted[T.d0 + j], slot = D.sslot[T.d0 + j];
        if (D.f[fi].tag > 255) continue; // a present one makes the table big
        o << "    if (e" << slot << " != 0xffffffffu) em.put_n(" << D.f[fi].tag << "u | ((uint64_t)__builtin_bswap16((uint16_t)e"
          << slot << ") << 8), 3);\n";
    }
    o << "  } else {\n";
    for (uint32_t j = 0; j < T.nd; j++) {
        const uint32_t fi = D.sorted[T.d0 + j], slot = D.sslot[T.d0 + j];
        o << "    if (e" << slot << " != 0xffffffffu) { em.be(" << D.f[fi].tag << "u, 2); em.be(e" << slot << ", 4); }\n";
    }
    o << "  }\n"
      << "  em.rvarint(data);\n  em.rvarint((uint64_t)nf * (big ? 6 : 3));\n"
      << "  em.put1(big ? T_BIG_MESSAGE : T_MESSAGE);\n  em.finish();\n";
}

// The generated Write() of a message table (internal/lang/generator/message.go:319-439,
// internal/writer/writer.go:376-553) for one row at start: every column read issued before the
// first byte is written, then the fields in write order (constant kinds, heaps and tags), the
// table in the Writer's tie-sorted order over the present fields, the trailer.  Sub-messages and
// list elements are children written by their tables' later launches into the gaps skipped here.
// the column reads of direct field k of table T issued before the first byte (values; a
// sub-message's or list's presence; a sub-message's size)
// (sfx / rv: the variables' suffix and the row expression, for a writer over two rows at once)
void gen_field_loads(std::ostringstream &o, const TreeDesc &D, const TTable &T, uint32_t k, bool eager, const char *ind,
                     const std::string &sfx = "", const std::string &rv = "row") {
    const TField &F = D.f[D.direct[T.d0 + k]];
    if ((F.kind >= spec::K_BOOL && F.kind <= spec::K_BYTES) || F.kind == spec::K_ANY) {
        if (eager)
            o << ind << "uint64_t a" << k << sfx << "[4];\n" << ind << "load_value_k<" << (int)F.kind << ">(" << col_expr(F.col)
              << ", " << rv << ", a" << k << sfx << ");\n";
    } else if (F.kind == spec::K_MESSAGE || F.kind == spec::K_LIST)
        o << ind << "const uint32_t pr" << k << sfx << " = ((const uint8_t *)" << col_expr(F.present) << ")[" << rv << "];\n";
    if (F.kind == spec::K_MESSAGE) o << ind << "const uint32_t sz" << k << sfx << " = B.size[" << F.table << "][" << rv << "];\n";
    // a struct's member values (every scalar member of its subtree: gen_struct_emit)
    if (F.kind == spec::K_STRUCT && eager) {
        const uint32_t fi = D.direct[T.d0 + k];
        for (uint32_t i = fi + 1; i < F.send; i++)
            if (D.f[i].kind != spec::K_STRUCT)
                o << ind << "uint64_t m" << i << sfx << "[4];\n" << ind << "load_value_k<" << (int)D.f[i].kind << ">("
                  << col_expr(D.f[i].col) << ", " << rv << ", m" << i << sfx << ");\n";
    }
    // a list's element range [begin[row], begin[row + 1]) (the size pass checked BEGIN)
    if (F.kind == spec::K_LIST)
        o << ind << "const uint32_t j0_" << k << sfx << " = ((const uint32_t *)" << col_expr(D.t[F.table].begin_col) << ")[" << rv
          << "], j1_" << k << sfx << " = ((const uint32_t *)" << col_expr(D.t[F.table].begin_col) << ")[" << rv << " + 1];\n";
}

// binds gen_field_loads' suffixed variables of field k to the names gen_field_write reads
void gen_field_bind(std::ostringstream &o, const TreeDesc &D, const TTable &T, uint32_t k, const std::string &sfx,
                    const char *ind) {
    const TField &F = D.f[D.direct[T.d0 + k]];
    if ((F.kind >= spec::K_BOOL && F.kind <= spec::K_BYTES) || F.kind == spec::K_ANY)
        o << ind << "uint64_t (&a" << k << ")[4] = a" << k << sfx << ";\n";
    else if (F.kind == spec::K_MESSAGE || F.kind == spec::K_LIST)
        o << ind << "const uint32_t pr" << k << " = pr" << k << sfx << ";\n";
    if (F.kind == spec::K_MESSAGE) o << ind << "const uint32_t sz" << k << " = sz" << k << sfx << ";\n";
    if (F.kind == spec::K_LIST)
        o << ind << "const uint32_t j0_" << k << " = j0_" << k << sfx << ", j1_" << k << " = j1_" << k << sfx << ";\n";
    if (F.kind == spec::K_STRUCT) {
        const uint32_t fi = D.direct[T.d0 + k];
        for (uint32_t i = fi + 1; i < F.send; i++)
            if (D.f[i].kind != spec::K_STRUCT) o << ind << "uint64_t (&m" << i << ")[4] = m" << i << sfx << ";\n";
    }
}

// struct field sf's EncodeXxxTo (internal/lang/generator/struct.go:115-142) from its loaded
// members m<i>: the members in declaration order (an inner struct is its own EncodeXxxTo in
// place), then EncodeStruct's rvarint(data size) | TypeStruct (tree_core.hpp emit_struct)
void gen_struct_emit(std::ostringstream &o, const TreeDesc &D, uint32_t sf, int d, const std::string &ind) {
    const TField &F = D.f[sf];
    o << ind << "{ const uint64_t ss" << d << " = em.pos;\n";
    for (uint32_t k = 0; k < F.nmem; k++) {
        const uint32_t mi = D.members[F.mem0 + k];
        const TField &M = D.f[mi];
        if (M.kind == spec::K_STRUCT) {
            gen_struct_emit(o, D, mi, d + 1, ind + "  ");
        } else {
            const bool heap = M.kind == spec::K_STRING || M.kind == spec::K_BYTES;
            o << ind << "  emit_value_k<" << (int)M.kind << ">(em, m" << mi << ", "
              << (heap ? "B.heaps[" + std::to_string(M.col) + "], B.heap_lens[" + std::to_string(M.col) + "]" : "nullptr, 0")
              << ");\n";
        }
    }
    o << ind << "  em.rvarint(em.pos - ss" << d << ");\n" << ind << "  em.put1(T_STRUCT);\n" << ind << "}\n";
}

// the size expression of a scalar value v (a loaded column element) of kind K (encode_core.hpp
// field_size rules)
std::string value_size_expr(int K, const std::string &v) {
    if (K == spec::K_BOOL) return "1";
    if (K == spec::K_BYTE) return "2";
    if (K == spec::K_INT16) return "(vlen32(zigzag32((int16_t)" + v + "[0])) + 1)";
    if (K == spec::K_INT32) return "(vlen32(zigzag32((int32_t)" + v + "[0])) + 1)";
    if (K == spec::K_INT64) return "(vlen64(zigzag64((int64_t)" + v + "[0])) + 1)";
    if (K == spec::K_UINT16 || K == spec::K_UINT32 || K == spec::K_UINT64) return "(vlen64(" + v + "[0]) + 1)";
    if (K == spec::K_FLOAT32) return "5";
    if (K == spec::K_FLOAT64 || K == spec::K_BIN64) return "9";
    if (K == spec::K_BIN128) return "17";
    if (K == spec::K_BIN256) return "33";
    const std::string len = "(uint64_t)(uint32_t)(" + v + "[0] >> 32)";
    if (K == spec::K_STRING) return "(" + len + " + vlen32((uint32_t)(" + v + "[0] >> 32)) + 2)";
    return "(" + len + " + vlen32((uint32_t)(" + v + "[0] >> 32)) + 1)"; // BYTES
}

// struct field sf's encoded size (tree_core.hpp struct_size) from its loaded members m<i>, into
// the variable `var` (declared here); a data size past MAX_SIZE sets err
void gen_struct_size(std::ostringstream &o, const TreeDesc &D, uint32_t sf, const std::string &var, const std::string &ind) {
    const TField &F = D.f[sf];
    o << ind << "uint64_t " << var << " = 0;\n" << ind << "{\n";
    for (uint32_t k = 0; k < F.nmem; k++) {
        const uint32_t mi = D.members[F.mem0 + k];
        const TField &M = D.f[mi];
        if (M.kind == spec::K_STRUCT) {
            gen_struct_size(o, D, mi, var + "_" + std::to_string(k), ind + "  ");
            o << ind << "  " << var << " += " << var << "_" << k << ";\n";
        } else {
            o << ind << "  " << var << " += " << value_size_expr(M.kind, "m" + std::to_string(mi)) << ";\n";
            if (M.kind == spec::K_STRING || M.kind == spec::K_BYTES)
                o << ind << "  { const uint32_t off = (uint32_t)m" << mi << "[0], len = (uint32_t)(m" << mi << "[0] >> 32);\n"
                  << ind << "    if ((uint64_t)len > MAX_SIZE || (uint64_t)off + len > B.heap_lens[" << M.col << "]) err = true; }\n";
        }
    }
    o << ind << "  if (" << var << " > MAX_SIZE) err = true;\n"
      << ind << "  " << var << " += vlen64(" << var << ") + 1;\n" << ind << "}\n";
}

// direct field k of table T in write order: its bytes through em (children: the gaps they fill,
// their rows' positions), then its end mark (e<k> or ends_[k] = em.pos - start), nf, bigtag
void gen_field_write(std::ostringstream &o, const TreeDesc &D, const TTable &T, uint32_t k, bool eager) {
    const uint32_t fi = D.direct[T.d0 + k];
    const TField &F = D.f[fi];
    auto load = [&](const char *ind) {
        o << ind << "uint64_t a" << k << "[4];\n" << ind << "load_value_k<" << (int)F.kind << ">(" << col_expr(F.col)
          << ", row, a" << k << ");\n";
    };
    const std::string ev = eager ? "e" + std::to_string(k) : "ends_[" + std::to_string(k) + "]";
    const std::string mark = "    " + ev + " = (uint32_t)(em.pos - start);\n    nf++;\n" +
                             (F.tag > 255 ? "    bigtag = true;\n" : "");
    if (eager) o << "  uint32_t e" << k << " = 0xffffffffu; // field " << fi << " tag " << F.tag << "\n";
    else o << "  ends_[" << k << "] = 0xffffffffu; // field " << fi << " tag " << F.tag << "\n";
    if (F.kind >= spec::K_BOOL && F.kind <= spec::K_BYTES) {
        const bool heap = F.kind == spec::K_STRING || F.kind == spec::K_BYTES;
        o << "  {\n";
        if (!eager) load("    ");
        o << "    emit_value_k<" << (int)F.kind << ">(em, a" << k << ", "
          << (heap ? "B.heaps[" + std::to_string(F.col) + "], B.heap_lens[" + std::to_string(F.col) + "]" : "nullptr, 0")
          << ");\n" << mark << "  }\n";
    } else if (F.kind == spec::K_ANY) {
        if (!eager) load("  ");
        o << "  if ((uint32_t)(a" << k << "[0] >> 32)) {\n    emit_value_k<" << (int)F.kind << ">(em, a" << k
          << ", B.heaps[" << F.col << "], B.heap_lens[" << F.col << "]);\n" << mark << "  }\n";
    } else if (F.kind == spec::K_STRUCT) {
        if (eager) gen_struct_emit(o, D, fi, 0, "  ");
        else o << "  emit_struct(em, B, D, " << fi << "u, row);\n";
        o << "  {\n" << mark << "  }\n";
    } else if (F.kind == spec::K_MESSAGE) {
        o << "  if (pr" << k << ") {\n    B.pos[" << F.table << "][row] = em.pos;\n    em.skip(sz" << k << ");\n" << mark
          << "  } else {\n    B.pos[" << F.table << "][row] = ~0ull; // absent: its row is not written\n  }\n";
    } else if (F.kind == spec::K_LIST) {
        const int y = F.table;
        o << "  if (!pr" << k << ") { // absent: rows in its range (if any) are not written\n"
          << "    for (uint32_t j = j0_" << k << "; j < j1_" << k << "; j++) B.pos[" << y << "][j] = ~0ull;\n  }\n";
        o << "  if (pr" << k << ") {\n"
          << "    emit_list(em, B, " << y << "u, j0_" << k << ", j1_" << k << ");\n"
          << mark << "  }\n";
    }
}

// The generated Write() of a message table (internal/lang/generator/message.go:319-439,
// internal/writer/writer.go:376-553) for one row at start: every column read issued before the
// first byte is written, then the fields in write order (constant kinds, heaps and tags), the
// table in the Writer's tie-sorted order over the present fields, the trailer.  Sub-messages and
// list elements are children written by their tables' later launches into the gaps skipped here.
void gen_write_table(std::ostringstream &o, const TreeDesc &D, uint32_t t) {
    const TTable &T = D.t[t];
    // a table of more than 64 direct fields loads each value where it is written (all of them in
    // flight at once would hold ~4 registers per field), and its writer is a function of its own:
    // inlined into the level-fused kernel, hiprtc spent minutes allocating registers over it
    const bool eager = T.nd <= 64;
    // (and out of line in a tree of many tables too: 114 writers inlined into the one level-fused
    // kernel took hiprtc 13 minutes)
    const bool inl = eager && D.ntables <= 32;
    o << "template <class E>\n__device__ " << (inl ? "__forceinline__" : "__noinline__") << " void gen_wrow_" << t
      << "(E &em, const TreeDesc &D, const TreeBufs &B, uint64_t row, uint64_t start) {\n";
    for (uint32_t k = 0; k < T.nd; k++) gen_field_loads(o, D, T, k, eager, "  ");
    o << "  uint32_t nf = 0;\n  bool bigtag = false;\n";
    // field ends: registers (e<k>), or for a wide table an array the table loop reads at run time
    if (!eager) o << "  uint32_t ends_[" << T.nd << "];\n";
    for (uint32_t k = 0; k < T.nd; k++) gen_field_write(o, D, T, k, eager);
    // IsBigMessage (internal/format/msg.go:43-61), the table (encode/msg.go:58-72), the trailer
    o << "  const uint64_t data = em.pos - start;\n"
      << "  const bool big = bigtag || (nf > 0 && data > 65535);\n";
    if (!eager) {
        // the wide table's entries in a run-time loop over the Writer's order (tree.hip layout:
        // sorted[], sslot[]): a third of the unrolled code
        o << "  for (uint32_t j = 0; j < " << T.nd << "u; j++) {\n"
          << "    const uint32_t e = ends_[D.sslot[" << T.d0 << "u + j]];\n"
          << "    if (e == 0xffffffffu) continue;\n"
          << "    const uint32_t tag = D.f[D.sorted[" << T.d0 << "u + j]].tag;\n"
          << "    if (!big) em.put_n(tag | ((uint64_t)__builtin_bswap16((uint16_t)e) << 8), 3);\n"
          << "    else { em.be(tag, 2); em.be(e, 4); }\n  }\n"
          << "  em.rvarint(data);\n  em.rvarint((uint64_t)nf * (big ? 6 : 3));\n"
          << "  em.put1(big ? T_BIG_MESSAGE : T_MESSAGE);\n  em.finish();\n}\n";
    } else {
        gen_table_trailer(o, D, T);
        o << "}\n";
    }
    // a row no owner placed (its own owner absent or unplaced): its children are not written either
    o << "__device__ __forceinline__ void gen_unplace_" << t << "(const TreeDesc &D, const TreeBufs &B, uint64_t row) {\n";
    for (uint32_t k = 0; k < T.nd; k++) {
        const TField &F = D.f[D.direct[T.d0 + k]];
        if (F.kind == spec::K_MESSAGE) {
            o << "  B.pos[" << F.table << "][row] = ~0ull;\n";
        } else if (F.kind == spec::K_LIST) {
            o << "  { bool lerr = false; uint32_t j0, j1; list_span(B, D, " << F.table << "u, row, j0, j1, lerr);\n"
              << "    for (uint32_t j = j0; j < j1; j++) B.pos[" << F.table << "][j] = ~0ull; }\n";
        }
    }
    o << "}\n";
}

bool tree_tile(const TreeDesc &D);
void tile_cuts(const TreeDesc &D, uint32_t *cut);

// The generated writer's size pass for a message table (tree.hip tree_size_kernel with constant
// kinds, columns and tags): every column read first, then the encoded sizes, IsBigMessage.
void gen_size_table(std::ostringstream &o, const TreeDesc &D, uint32_t t) {
    const TTable &T = D.t[t];
    o << "__device__ __forceinline__ void gen_srow_" << t
      << "(const TreeDesc &D, const TreeBufs &B, uint32_t x, uint64_t row, bool &err) {\n"
      << "  {\n";
    for (uint32_t k = 0; k < T.nd; k++) {
        const TField &F = D.f[D.direct[T.d0 + k]];
        if ((F.kind >= spec::K_BOOL && F.kind <= spec::K_BYTES) || F.kind == spec::K_ANY)
            o << "    uint64_t a" << k << "[4];\n    load_value_k<" << (int)F.kind << ">(" << col_expr(F.col) << ", row, a" << k
              << ");\n";
        else if (F.kind == spec::K_MESSAGE || F.kind == spec::K_LIST)
            o << "    const uint32_t pr" << k << " = ((const uint8_t *)" << col_expr(F.present) << ")[row];\n";
        if (F.kind == spec::K_STRUCT) gen_field_loads(o, D, T, k, true, "    ");
        if (F.kind == spec::K_LIST)
            o << "    const uint32_t j0_" << k << " = ((const uint32_t *)" << col_expr(D.t[F.table].begin_col) << ")[row], j1_" << k
              << " = ((const uint32_t *)" << col_expr(D.t[F.table].begin_col) << ")[row + 1];\n";
    }
    // the records' table under the record-tile writer (gen_tile): also each field block's end
    // offset (B.tblk, inclusive prefix over the blocks) and the present direct fields (B.tmask)
    const bool tile = t == 0 && tree_tile(D);
    uint32_t cut[spec::TREE_TILE_W + 1];
    if (tile) tile_cuts(D, cut);
    o << "    uint64_t data = 0;\n    uint32_t nf = 0;\n    bool bigtag = false;\n"
      << (tile ? "    uint64_t bm = 0;\n" : "");
    for (uint32_t k = 0; k < T.nd; k++) {
        const uint32_t fi = D.direct[T.d0 + k];
        const TField &F = D.f[fi];
        const std::string tg = (F.tag > 255 ? " bigtag = true;" : "") +
                               (tile ? " bm |= 1ull << " + std::to_string(k) + ";" : std::string());
        for (int bl = 0; tile && bl < spec::TREE_TILE_W; bl++) // blocks ending before field k
            if (cut[bl + 1] == k) o << "    const uint64_t tb" << bl << " = data;\n";
        switch (F.kind) {
        case spec::K_MESSAGE:
            o << "    if (pr" << k << ") { data += B.size[" << F.table << "][row]; nf++;" << tg << " }\n";
            break;
        case spec::K_LIST:
            o << "    if (pr" << k << ") { data += list_total(B, " << F.table << "u, j0_" << k << ", j1_" << k << ", err); nf++;" << tg
              << " }\n";
            break;
        case spec::K_STRUCT:
            gen_struct_size(o, D, fi, "st" + std::to_string(k), "    ");
            o << "    data += st" << k << "; nf++;" << tg << "\n";
            break;
        case spec::K_ANY:
            o << "    { const uint32_t off = (uint32_t)a" << k << "[0], len = (uint32_t)(a" << k << "[0] >> 32);\n"
              << "      if ((uint64_t)len > MAX_SIZE || (uint64_t)off + len > B.heap_lens[" << F.col << "]) err = true;\n"
              << "      if (len) { data += len; nf++;" << tg << " } }\n";
            break;
        case spec::K_STRING:
        case spec::K_BYTES:
            o << "    { const uint32_t off = (uint32_t)a" << k << "[0], len = (uint32_t)(a" << k << "[0] >> 32);\n"
              << "      if ((uint64_t)len > MAX_SIZE || (uint64_t)off + len > B.heap_lens[" << F.col << "]) err = true;\n"
              << "      data += (uint64_t)len + vlen32(len) + " << (F.kind == spec::K_STRING ? 2 : 1) << "; nf++;" << tg << " }\n";
            break;
        default: {
            const int K = F.kind;
            std::string sz;
            if (K == spec::K_BOOL) sz = "1";
            else if (K == spec::K_BYTE) sz = "2";
            else if (K == spec::K_INT16) sz = "vlen32(zigzag32((int16_t)a" + std::to_string(k) + "[0])) + 1";
            else if (K == spec::K_INT32) sz = "vlen32(zigzag32((int32_t)a" + std::to_string(k) + "[0])) + 1";
            else if (K == spec::K_INT64) sz = "vlen64(zigzag64((int64_t)a" + std::to_string(k) + "[0])) + 1";
            else if (K == spec::K_UINT16 || K == spec::K_UINT32 || K == spec::K_UINT64)
                sz = "vlen64(a" + std::to_string(k) + "[0]) + 1";
            else if (K == spec::K_FLOAT32) sz = "5";
            else if (K == spec::K_FLOAT64 || K == spec::K_BIN64) sz = "9";
            else if (K == spec::K_BIN128) sz = "17";
            else sz = "33";
            o << "    data += " << sz << "; nf++;" << tg << "\n";
        }
        }
    }
    if (tile) {
        for (int bl = 0; bl < spec::TREE_TILE_W; bl++)
            if (cut[bl + 1] == T.nd) o << "    const uint64_t tb" << bl << " = data;\n";
        for (int bl = 0; bl < spec::TREE_TILE_W; bl++) o << "    B.tblk[row * " << spec::TREE_TILE_W << " + " << bl << "] = (uint32_t)tb" << bl << ";\n";
        o << "    B.tmask[row] = bm;\n";
    }
    // IsBigMessage (internal/format/msg.go:43-61), encodeMessageTable sizes
    o << "    const bool big = bigtag || (nf > 0 && data > 65535);\n"
      << "    const uint64_t tsize = (uint64_t)nf * (big ? 6 : 3);\n"
      << "    if (data > MAX_SIZE) err = true;\n"
      << "    const uint64_t total = data + tsize + vlen64(data) + vlen64(tsize) + 1;\n"
      << "    if (total > 0xffffffffull) err = true;\n"
      << "    B.size[x][row] = (uint32_t)total;\n"
      << "  }\n}\n";
}

// The sub-message tables of group root x after its root table's code, each over the range its
// owner field left in its slot; a sub-table whose trailer is invalid sets its owner field's *Err
// bit (the owner's getter would have failed on the same trailer): on a wave group's root through
// ro (pair), else into the owner's ERRMASK column, which the owner's code stored before.
void gen_sub_tables(std::ostringstream &o, const TreeDesc &D, uint32_t x, int pair_w, const uint32_t *tw,
                    const std::string &fb) {
    const TTable &T = D.t[x];
    for (uint32_t g = 1; g < T.gn; g++) {
        const uint32_t y = D.group[T.g0 + g];
        if (pair_w >= 0 && tw[y] != (uint32_t)pair_w) continue;
        const TTable &Y = D.t[y], &Pt = D.t[Y.parent];
        std::string bad;
        uint32_t k = 0;
        while (k < Pt.nd && D.direct[Pt.d0 + k] != Y.field) k++;
        if (Pt.err_col >= 0 && k < 64) {
            const std::string bit = "(1ull << " + std::to_string(k) + ")";
            bad = pair_w >= 0 && Y.parent == x ? "ro.errs |= " + bit + ";"
                                               : "((uint64_t *)" + col_expr(Pt.err_col) + ")[row] |= " + bit + ";";
        }
        const std::string r = "gr[" + std::to_string(Y.gslot) + " * 64]";
        gen_message_table(o, D, y, "(long long)" + r + ".x", "(long long)" + r + ".y", false, nullptr, fb, bad);
    }
}

// ---- the root group on a wave pair (tree_decode_core.hpp tree_rows_pair) ----
// A cost per field, about its LDS reads and VALU: the pair split balances these.
uint32_t tree_table_cost(const TreeDesc &D, uint32_t t);
uint32_t tree_field_cost(const TreeDesc &D, uint32_t fi) {
    const TField &F = D.f[fi];
    switch (F.kind) {
    case spec::K_STRING: case spec::K_BYTES: case spec::K_BIN128: case spec::K_BIN256: return 3;
    case spec::K_STRUCT: return 2 + 2 * (F.send - fi - 1);
    case spec::K_ANY: return 5;
    case spec::K_LIST: return 5;
    case spec::K_MESSAGE: return 3 + tree_table_cost(D, F.table);
    default: return 2;
    }
}
uint32_t tree_table_cost(const TreeDesc &D, uint32_t t) {
    const TTable &T = D.t[t];
    uint32_t c = 4;
    for (uint32_t k = 0; k < T.nd; k++) c += tree_field_cost(D, D.direct[T.d0 + k]);
    return c;
}

// Group root x split over P waves: sel[w][k] = wave w decodes root field k (with the sub-message
// tables below it, which need the range it finds).  Heaviest first, each to the least loaded
// wave.  false when the root has too few fields to split.
bool pair_split(const TreeDesc &D, uint32_t x, int P, std::vector<char> *sel, uint32_t *table_wave) {
    const TTable &T = D.t[x];
    if (T.shape != spec::SHAPE_MESSAGE || T.nd < (uint32_t)(2 * P)) return false;
    std::vector<uint32_t> ks(T.nd);
    for (uint32_t k = 0; k < T.nd; k++) ks[k] = k;
    std::stable_sort(ks.begin(), ks.end(), [&](uint32_t a, uint32_t b) {
        return tree_field_cost(D, D.direct[T.d0 + a]) > tree_field_cost(D, D.direct[T.d0 + b]);
    });
    uint32_t load[4] = {0, 0, 0, 0};
    for (int w = 0; w < P; w++) sel[w].assign(T.nd, 0);
    for (uint32_t k : ks) {
        int w = 0;
        for (int v = 1; v < P; v++)
            if (load[v] < load[w]) w = v;
        sel[w][k] = 1;
        load[w] += tree_field_cost(D, D.direct[T.d0 + k]);
    }
    for (uint32_t g = 1; g < T.gn; g++) {
        const uint32_t y = D.group[T.g0 + g];
        uint32_t a = y;
        while (D.t[a].parent != x) a = D.t[a].parent;
        table_wave[y] = 0;
        for (uint32_t k = 0; k < T.nd; k++)
            if (D.direct[T.d0 + k] == D.t[a].field)
                for (int w = 0; w < P; w++)
                    if (sel[w][k]) table_wave[y] = (uint32_t)w;
    }
    return true;
}

// spec_tree_group_<x>p<P>: the group's row code split over P waves (pair_split).  The waves
// share one set of range slots: a sub-message table's slot is written and read by the wave that
// owns it (a row on the run-time path has every wave write every slot, with the same values).
void gen_pair_rows(std::ostringstream &o, const TreeDesc &D, uint32_t x, int P) {
    std::vector<char> sel[4];
    uint32_t tw[spec::TREE_MAX_T] = {};
    if (!pair_split(D, x, P, sel, tw)) return;
    const TTable &T = D.t[x];
    const std::string fn = "gen_pair_" + std::to_string(x) + "_" + std::to_string(P) + "_w";
    for (int w = 0; w < P; w++) {
        o << "template <class Src>\n__device__ __forceinline__ void " << fn << w
          << "(const Src &s, const TreeDesc &D, const TreeBufs &B, uint64_t row, long long lo, long long hi, uint2 *gr, "
             "RowOut &ro) {\n";
        const std::string fb = "tree_message_fallback_p<" + std::to_string(P) + ">";
        gen_message_table(o, D, x, "lo", "hi", true, &sel[w], fb);
        gen_sub_tables(o, D, x, w, tw, fb);
        o << "}\n";
    }
    std::ostringstream call;
    call << "      switch (threadIdx.x >> 6) {\n";
    for (int w = 0; w < P; w++)
        call << "      case " << w << ": " << fn << w << "(s, D, B, row, lo, hi, gr, ro); break;\n";
    call << "      default: break;\n      }\n";
    // P waves of one block per SIMD... and as many blocks per CU as the LDS holds (four for
    // pkg1): registers for 8 / 4 waves per SIMD-pair budget -> at most 512 / P VGPRs
    o << "extern \"C\" __global__ __launch_bounds__(" << 64 * P << ") __attribute__((amdgpu_waves_per_eu(" << P
      << "))) void spec_tree_group_" << x << "p" << P
      << "(const TreeDesc *Dp, const TreeBufs *Bp, uint32_t x, uint32_t slab, uint32_t slots, uint32_t rpw) {\n"
      << "  const TreeDesc &D = *Dp;\n"
      << "  const TreeBufs &B = *Bp;\n"
      << "  const uint64_t rows = dec_rows(D, B, x);\n"
      << "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
      << "  uint2 *gr = (uint2 *)(smem + slab) + (threadIdx.x & 63);\n"
      << "  uint4 *xch = (uint4 *)(smem + slab + slots);\n"
      << "  (void)rpw;\n"
      << "  tree_rows_pair<" << P << ">(B, x, rows, slab, xch,\n"
      << "    [&](const TreeLds &s, uint64_t row, long long lo, long long hi, RowOut &ro) {\n"
      << call.str() << "    },\n"
      << "    [&](const GlobalSrc &s, uint64_t row, long long lo, long long hi, RowOut &ro) {\n"
      << call.str() << "    },\n"
      << "    [&](uint64_t row, bool panic, const RowOut &a, const RowOut &b) {\n"
      << "      uint64_t *errp = " << (T.err_col >= 0 ? "(uint64_t *)" + col_expr(T.err_col) : std::string("nullptr")) << ";\n"
      << "      if (a.fast && errp) errp[row] = a.errs | b.errs;\n"
      << "      const uint32_t st = a.st == ST_PANIC || b.st == ST_PANIC ? (uint32_t)ST_PANIC : a.st;\n"
      << "      store_u8(" << col_expr(T.status_col) << ", row, panic ? (uint32_t)ST_PANIC : st);\n"
      << "    });\n"
      << "}\n";
}

// ---- the record-tile writer (tree_core.hpp MkL, tile_copy_out) ----
// spec_tree_write_tile: one workgroup of TILE_W waves per 64 consecutive records.  Depth 0: the
// records' direct fields are split into TILE_W contiguous blocks, wave w writing block w of all
// 64 records (so a wave runs one block's code, no divergence) at the block's offset, which the
// size pass left per record with the record's present fields (B.tblk, B.tmask), and their table
// entries at (popcount of the present fields before them in the Writer's order); the last wave
// writes the trailer.  Depth d > 0: the tile's rows of every table at depth d (a
// contiguous row range per table, from the records' range through BEGIN columns) over all lanes,
// through the tables' generated writers.  A barrier between depths (children placed by their
// owners).  Everything goes to an LDS image of the tile's output range, stored once with 16-byte
// stores; the bytes of a range longer than the image past its first cap bytes are stored straight
// to HBM (a loop of passes over windows of the range tripled the kernel's compile time).
constexpr int TILE_W = spec::TREE_TILE_W;

bool tree_tile(const TreeDesc &D) {
    if (!SPEC_AB_TREE_TILE || D.ntables > 32 || D.t[0].shape != spec::SHAPE_MESSAGE) return false;
    for (uint32_t t = 0; t < D.ntables; t++)
        if (D.t[t].shape == spec::SHAPE_MESSAGE && D.t[t].nd > 64) return false;
    return true;
}

// a records' field's share of its wave's time in the tile writer, in scalar fields (fitted to the
// per-wave clocks of a -DSPEC_AB_TILE_CLOCK=1 build on pkg1: a list ≈ 5, a string ≈ 2)
uint32_t tile_field_cost(const TreeDesc &D, const TField &F) {
    switch (F.kind) {
    case spec::K_STRING: case spec::K_BYTES: case spec::K_ANY: return 2;
    case spec::K_BIN128: return 2;
    case spec::K_BIN256: return 3;
    case spec::K_STRUCT: return 1 + (F.send - 1u - (uint32_t)(&F - D.f));
    case spec::K_LIST: return 5;
    case spec::K_MESSAGE: return 1;
    default: return 1;
    }
}

// the records' direct fields in TILE_W contiguous blocks of about equal cost: block b is
// [cut[b], cut[b + 1])
void tile_cuts(const TreeDesc &D, uint32_t *cut) {
    const TTable &T = D.t[0];
    std::vector<uint32_t> cost(T.nd);
    uint32_t total = 0;
    for (uint32_t k = 0; k < T.nd; k++) total += cost[k] = tile_field_cost(D, D.f[D.direct[T.d0 + k]]);
    uint32_t k = 0, acc = 0;
    cut[0] = 0;
    for (int b = 0; b < TILE_W; b++) {
        // fields while below the block's share of the total, the last one only if that lands closer
        const int64_t target = (int64_t)total * (b + 1) / TILE_W;
        while (k < T.nd && (b == TILE_W - 1 || ((int64_t)acc < target &&
                                                 (int64_t)(acc + cost[k]) - target <= target - (int64_t)acc)))
            acc += cost[k++];
        cut[b + 1] = k;
    }
    cut[TILE_W] = T.nd;
}

// A table whose tile rows at one depth run in ROUNDS (SPEC_AB_TILE_ROUNDS): each thread issues the
// reads of its next row of every such table at once, then writes them one after another — a
// thread holds about one row per table per tile, so per-table loops were one dependent chain of
// reads per table.  Message tables, lists of scalars / strings / bytes, lists of structs.
bool tile_round_ok(const TreeDesc &D, uint32_t x) {
    const TTable &X = D.t[x];
    if (!SPEC_AB_TILE_ROUNDS) return false;
    if (X.shape == spec::SHAPE_MESSAGE || X.shape == spec::SHAPE_STRUCT) return true;
    return X.shape == spec::SHAPE_VALUE && D.f[X.field].elem >= spec::K_BOOL && D.f[X.field].elem <= spec::K_BYTES;
}

// the reads of row `rv` of table x (round mode) into variables suffixed sfx: declarations
// (zeroed) into decl, the reads, under the row's validity, into rd
void gen_round_loads(std::ostringstream &decl, std::ostringstream &rd, const TreeDesc &D, uint32_t x,
                     const std::string &sfx, const std::string &rv) {
    const TTable &X = D.t[x];
    auto member_loads = [&](uint32_t sf) {
        for (uint32_t i = sf + 1u; i < D.f[sf].send; i++)
            if (D.f[i].kind != spec::K_STRUCT) {
                decl << "    uint64_t m" << i << sfx << "[4] = {0, 0, 0, 0};\n";
                rd << "      load_value_k<" << (int)D.f[i].kind << ">(" << col_expr(D.f[i].col) << ", " << rv << ", m" << i << sfx
                   << ");\n";
            }
    };
    decl << "    uint64_t start" << sfx << " = ~0ull;\n";
    rd << "      start" << sfx << " = B.pos[" << x << "][" << rv << "];\n";
    if (X.shape == spec::SHAPE_VALUE) {
        const TField &F = D.f[X.field];
        decl << "    uint64_t a" << sfx << "[4] = {0, 0, 0, 0};\n";
        rd << "      load_value_k<" << (int)F.elem << ">(" << col_expr(F.col) << ", " << rv << ", a" << sfx << ");\n";
        return;
    }
    if (X.shape == spec::SHAPE_STRUCT) {
        member_loads(X.field);
        return;
    }
    for (uint32_t k = 0; k < X.nd; k++) {
        const uint32_t fi = D.direct[X.d0 + k];
        const TField &F = D.f[fi];
        const std::string ks = std::to_string(k);
        if ((F.kind >= spec::K_BOOL && F.kind <= spec::K_BYTES) || F.kind == spec::K_ANY) {
            decl << "    uint64_t a" << k << sfx << "[4] = {0, 0, 0, 0};\n";
            rd << "      load_value_k<" << (int)F.kind << ">(" << col_expr(F.col) << ", " << rv << ", a" << k << sfx << ");\n";
        } else if (F.kind == spec::K_MESSAGE || F.kind == spec::K_LIST) {
            decl << "    uint32_t pr" << k << sfx << " = 0;\n";
            rd << "      pr" << k << sfx << " = ((const uint8_t *)" << col_expr(F.present) << ")[" << rv << "];\n";
        }
        if (F.kind == spec::K_MESSAGE) {
            decl << "    uint32_t sz" << k << sfx << " = 0;\n";
            rd << "      sz" << k << sfx << " = B.size[" << F.table << "][" << rv << "];\n";
        }
        if (F.kind == spec::K_LIST) {
            const std::string bc = "((const uint32_t *)" + col_expr(D.t[F.table].begin_col) + ")";
            decl << "    uint32_t j0_" << k << sfx << " = 0, j1_" << k << sfx << " = 0;\n";
            rd << "      j0_" << k << sfx << " = " << bc << "[" << rv << "];\n      j1_" << k << sfx << " = " << bc << "[" << rv
               << " + 1];\n";
        }
        if (F.kind == spec::K_STRUCT) member_loads(fi);
    }
}

// the write of the row read by gen_round_loads (valid, placed)
void gen_round_write(std::ostringstream &o, const TreeDesc &D, uint32_t x, const std::string &sfx, const std::string &rv) {
    const TTable &X = D.t[x];
    o << "      {\n      const uint64_t row = " << rv << ", start = start" << sfx << ";\n      (void)row;\n";
    if (X.shape == spec::SHAPE_VALUE) {
        const TField &F = D.f[X.field];
        const bool heap = F.elem == spec::K_STRING || F.elem == spec::K_BYTES;
        o << "      if (start != ~0ull) {\n      auto em = mk(start);\n      emit_value_k<" << (int)F.elem << ">(em, a" << sfx << ", "
          << (heap ? "B.heaps[" + std::to_string(F.col) + "], B.heap_lens[" + std::to_string(F.col) + "]" : "nullptr, 0")
          << ");\n      em.finish();\n      }\n      }\n";
        return;
    }
    if (X.shape == spec::SHAPE_STRUCT) {
        for (uint32_t i = X.field + 1u; i < D.f[X.field].send; i++)
            if (D.f[i].kind != spec::K_STRUCT) o << "      uint64_t (&m" << i << ")[4] = m" << i << sfx << ";\n";
        o << "      if (start != ~0ull) {\n      auto em = mk(start);\n";
        gen_struct_emit(o, D, X.field, 0, "      ");
        o << "      em.finish();\n      }\n      }\n";
        return;
    }
    for (uint32_t k = 0; k < X.nd; k++) gen_field_bind(o, D, X, k, sfx, "      ");
    o << "      if (start == ~0ull) {\n        gen_unplace_" << x << "(D, B, row);\n      } else {\n"
      << "      auto em = mk(start);\n      uint32_t nf = 0;\n      bool bigtag = false;\n";
    for (uint32_t k = 0; k < X.nd; k++) gen_field_write(o, D, X, k, true);
    o << "  const uint64_t data = em.pos - start;\n  const bool big = bigtag || (nf > 0 && data > 65535);\n";
    gen_table_trailer(o, D, X);
    o << "      }\n      }\n";
}

void gen_tile(std::ostringstream &o, const TreeDesc &D) {
    const TTable &T = D.t[0];
    uint32_t cut[TILE_W + 1];
    tile_cuts(D, cut);
    // PRE[k]: the direct fields before k in the Writer's table order; BIGM: tags past 255
    std::vector<uint64_t> pre(T.nd, 0);
    uint64_t bigm = 0, seen = 0;
    for (uint32_t j = 0; j < T.nd; j++) {
        const uint32_t slot = D.sslot[T.d0 + j];
        pre[slot] = seen;
        seen |= 1ull << slot;
    }
    for (uint32_t k = 0; k < T.nd; k++)
        if (D.f[D.direct[T.d0 + k]].tag > 255) bigm |= 1ull << k;
    // block b of a record: its offset and the record's data size and present fields from the size
    // pass (gen_size_table: B.tblk, B.tmask), so the waves need not meet before writing
    for (int b = 0; b < TILE_W; b++) {
        o << "template <class Mk>\n__device__ __forceinline__ void gen_troot_" << b
          << "(const Mk &mk, const TreeDesc &D, const TreeBufs &B, uint64_t row) {\n"
          << "  const uint64_t start = B.offsets[row];\n"
          << "  const uint64_t off = " << (b ? "B.tblk[row * " + std::to_string(TILE_W) + " + " + std::to_string(b - 1) + "]" : "0")
          << ", data = B.tblk[row * " << TILE_W << " + " << TILE_W - 1 << "];\n"
          << "  const uint64_t m = B.tmask[row];\n";
        for (uint32_t k = cut[b]; k < cut[b + 1]; k++) gen_field_loads(o, D, T, k, true, "  ");
        if (b == 0) o << "  if (B.ends_out) B.ends_out[row] = start + B.size[0][row];\n";
        o << "  const bool big = (m & 0x" << std::hex << bigm << std::dec << "ull) != 0 || (m != 0 && data > 65535);\n"
          << "  auto em = mk(start + off);\n  uint32_t nf = 0;\n  bool bigtag = false;\n";
        for (uint32_t k = cut[b]; k < cut[b + 1]; k++) gen_field_write(o, D, T, k, true);
        o << "  em.finish();\n  const uint64_t tb = start + data;\n";
        for (uint32_t k = cut[b]; k < cut[b + 1]; k++) {
            const uint32_t tag = D.f[D.direct[T.d0 + k]].tag;
            o << "  if (e" << k << " != 0xffffffffu) {\n"
              << "    const uint64_t p = tb + (big ? 6u : 3u) * (uint32_t)__popcll(m & 0x" << std::hex << pre[k] << std::dec
              << "ull);\n"
              << "    if (!big) em.put_at(p, " << (tag & 0xff) << "u | ((uint64_t)__builtin_bswap16((uint16_t)e" << k
              << ") << 8), 3);\n"
              << "    else em.put_at(p, " << (((tag & 0xff) << 8) | (tag >> 8)) << "u | ((uint64_t)__builtin_bswap32(e" << k
              << ") << 16), 6);\n  }\n";
        }
        if (b == TILE_W - 1)
            o << "  { const uint32_t nt = (uint32_t)__popcll(m) * (big ? 6u : 3u);\n"
              << "    auto tr = mk(tb + nt);\n    tr.rvarint(data);\n    tr.rvarint(nt);\n"
              << "    tr.put1(big ? T_BIG_MESSAGE : T_MESSAGE);\n    tr.finish(); }\n";
        o << "  (void)nf; (void)bigtag;\n}\n";
    }
    // the rows of tables 1.. at their placed positions: a message row's column reads and its
    // position issued together (one round trip), the position checked after them
    for (uint32_t x = 1; x < D.ntables; x++) {
        const TTable &X = D.t[x];
        o << "template <class Mk>\n__device__ __forceinline__ void gen_trow_" << x
          << "(const Mk &mk, const TreeDesc &D, const TreeBufs &B, uint64_t row) {\n";
        if (X.shape == spec::SHAPE_MESSAGE) {
            for (uint32_t k = 0; k < X.nd; k++) gen_field_loads(o, D, X, k, true, "  ");
            o << "  const uint64_t start = B.pos[" << x << "][row];\n"
              << "  if (start == ~0ull) { gen_unplace_" << x << "(D, B, row); return; }\n"
              << "  auto em = mk(start);\n  uint32_t nf = 0;\n  bool bigtag = false;\n";
            for (uint32_t k = 0; k < X.nd; k++) gen_field_write(o, D, X, k, true);
            o << "  const uint64_t data = em.pos - start;\n"
              << "  const bool big = bigtag || (nf > 0 && data > 65535);\n";
            gen_table_trailer(o, D, X);
        } else if (X.shape == spec::SHAPE_VALUE && D.f[X.field].elem >= spec::K_BOOL && D.f[X.field].elem <= spec::K_BYTES) {
            const TField &F = D.f[X.field];
            const bool heap = F.elem == spec::K_STRING || F.elem == spec::K_BYTES;
            o << "  uint64_t a[4];\n  load_value_k<" << (int)F.elem << ">(" << col_expr(F.col) << ", row, a);\n"
              << "  const uint64_t start = B.pos[" << x << "][row];\n  if (start == ~0ull) return;\n"
              << "  auto em = mk(start);\n  emit_value_k<" << (int)F.elem << ">(em, a, "
              << (heap ? "B.heaps[" + std::to_string(F.col) + "], B.heap_lens[" + std::to_string(F.col) + "]" : "nullptr, 0")
              << ");\n  em.finish();\n";
        } else if (X.shape == spec::SHAPE_STRUCT) { // a list of structs: the element's EncodeXxxTo
            const TField &F = D.f[X.field];
            for (uint32_t i = X.field + 1u; i < F.send; i++)
                if (D.f[i].kind != spec::K_STRUCT)
                    o << "  uint64_t m" << i << "[4];\n  load_value_k<" << (int)D.f[i].kind << ">(" << col_expr(D.f[i].col)
                      << ", row, m" << i << ");\n";
            o << "  const uint64_t start = B.pos[" << x << "][row];\n  if (start == ~0ull) return;\n"
              << "  auto em = mk(start);\n";
            gen_struct_emit(o, D, X.field, 0, "  ");
            o << "  em.finish();\n";
        } else {
            o << "  const uint64_t start = B.pos[" << x << "][row];\n  if (start == ~0ull) return;\n"
              << "  auto em = mk(start);\n  emit_row_shaped(em, D, B, " << x << "u, row);\n";
        }
        o << "}\n";
    }
    int depth[spec::TREE_MAX_T] = {0}, maxd = 0;
    for (uint32_t x = 1; x < D.ntables; x++) {
        depth[x] = depth[D.t[x].parent] + 1;
        maxd = std::max(maxd, depth[x]);
    }
    o << "template <class Mk>\n__device__ __forceinline__ void gen_tile_body(const Mk &mk, const TreeDesc &D, const TreeBufs &B, "
         "uint64_t r0, uint64_t r1) {\n"
      << "  const uint64_t row = r0 + (threadIdx.x & 63);\n"
      << (SPEC_AB_TILE_CLOCK ? "  const uint64_t c0 = wall_clock64();\n" : "")
      << "  if (row < r1) switch (threadIdx.x >> 6) {\n";
    for (int b = 0; b < TILE_W; b++) o << "  case " << b << ": gen_troot_" << b << "(mk, D, B, row); break;\n";
    o << "  }\n  __syncthreads();\n  const uint64_t lo0 = r0, hi0 = r1;\n";
    if (SPEC_AB_TILE_CLOCK) o << "  if (threadIdx.x == 0) { B.tmask[r0] = c0; B.tmask[r0 + 1] = wall_clock64(); }\n";
    for (uint32_t x = 1; x < D.ntables; x++) {
        const TTable &X = D.t[x];
        // (an owner range that is empty reads no BEGIN: the column may be absent then)
        if (X.rel == spec::REL_MANY)
            o << "  const bool ne" << x << " = hi" << X.parent << " > lo" << X.parent << ";\n"
              << "  const uint64_t lo" << x << " = ne" << x << " ? ((const uint32_t *)" << col_expr(X.begin_col) << ")[lo"
              << X.parent << "] : 0, hi" << x << " = ne" << x << " ? ((const uint32_t *)" << col_expr(X.begin_col) << ")[hi"
              << X.parent << "] : 0;\n";
        else
            o << "  const uint64_t lo" << x << " = lo" << X.parent << ", hi" << x << " = hi" << X.parent << ";\n";
    }
    // depth d: the tables' row ranges laid end to end, index i to thread i mod blockDim; the
    // tables of tile_round_ok in rounds (every such table's next row of this thread read at once),
    // the others in one loop per table over this thread's indices in its segment (an if-chain
    // over the tables inside one loop took the register coalescer minutes)
    for (int d = 1; d <= maxd; d++) {
        o << "  { // depth " << d << "\n    uint64_t base = 0;\n";
        std::vector<uint32_t> rt;
        for (uint32_t x = 1; x < D.ntables; x++)
            if (depth[x] == d) {
                o << "    const uint64_t c" << x << " = hi" << x << " - lo" << x << ", b" << x << " = base;\n    base += c" << x << ";\n";
                if (tile_round_ok(D, x)) rt.push_back(x);
                else
                    o << "    for (uint64_t i = (uint32_t)(threadIdx.x - b" << x << ") % blockDim.x; i < c" << x
                      << "; i += blockDim.x)\n      gen_trow_" << x << "(mk, D, B, lo" << x << " + i);\n";
            }
        if (!rt.empty()) {
            o << "    for (uint64_t r = 0;; r += blockDim.x) {\n";
            std::ostringstream decl, rd, wr;
            for (uint32_t x : rt) {
                const std::string sx = "_t" + std::to_string(x), rv = "rw" + std::to_string(x);
                o << "    const uint64_t j" << x << " = (uint32_t)(threadIdx.x - b" << x << ") % blockDim.x + r;\n"
                  << "    const bool v" << x << " = j" << x << " < c" << x << ";\n"
                  << "    const uint64_t " << rv << " = lo" << x << " + j" << x << ";\n";
                rd << "      if (v" << x << ") {\n";
                gen_round_loads(decl, rd, D, x, sx, rv);
                rd << "      }\n";
                wr << "      if (v" << x << ") \n";
                gen_round_write(wr, D, x, sx, rv);
            }
            o << "    if (!(false";
            for (uint32_t x : rt) o << " || v" << x;
            o << ")) break;\n" << decl.str() << rd.str() << wr.str() << "    }\n";
        }
        o << "    (void)base;\n  }\n  __syncthreads();\n";
        if (SPEC_AB_TILE_CLOCK) o << "  if (threadIdx.x == 0) B.tmask[r0 + " << d + 1 << "] = wall_clock64();\n";
    }
    o << "}\n"
      << "extern \"C\" __global__ __launch_bounds__(" << TILE_W * 64
      << ") __attribute__((amdgpu_waves_per_eu(" << spec::TREE_TILE_WPE
      << "))) void spec_tree_write_tile(const TreeDesc *Dp, const TreeBufs *Bp, "
         "uint32_t cap) {\n"
      << "  const TreeDesc &D = *Dp;\n  const TreeBufs &B = *Bp;\n"
      << "  if (!B.out || *B.err || *B.total > B.out_cap) return;\n"
      << "  const uint64_t n = B.rows[0], r0 = (uint64_t)blockIdx.x * 64;\n  if (r0 >= n) return;\n"
      << "  const uint64_t r1 = r0 + 64 < n ? r0 + 64 : n;\n"
      << "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
      << "  TileU8 *img = (TileU8 *)smem;\n"
      << "  const uint64_t org = B.offsets[r0], fin = B.offsets[r1 - 1] + B.size[0][r1 - 1];\n"
      // (out + sh 16-byte aligned: the image's chunks are the output's)
      << "  const uint64_t sh = org - (((unsigned long long)B.out + org) & 15);\n"
      << (SPEC_AB_TILE_OR ? "  tile_clear(img, fin - sh < cap ? (uint32_t)(fin - sh) : cap);\n  __syncthreads();\n" : "")
      << "  gen_tile_body(MkL{img, B.out, sh, cap}, D, B, r0, r1);\n"
      << "  tile_copy_out(B.out, img, sh, org, fin < sh + cap ? fin : sh + cap);\n"
      << (SPEC_AB_TILE_CLOCK ? "  __syncthreads();\n  if (threadIdx.x == 0) B.tmask[r0 + 63] = wall_clock64();\n" : "")
      << "}\n";
}

std::string generate_tree(const TreeDesc &D, bool *has) {
    std::ostringstream o;
    o << (SPEC_AB_TILE_OR ? "#define SPEC_TILE_OR 1\n" : "") << "#include \"tree_decode_core.hpp\"\nusing namespace spec;\n";
    for (uint32_t t = 0; t < D.ntables; t++)
        if (D.t[t].shape == spec::SHAPE_MESSAGE) {
            gen_write_table(o, D, t);
            gen_size_table(o, D, t);
        }
    // level-fused launches (tree_core.hpp TableSet): blockIdx.y = the set's table
    o << "extern \"C\" __global__ __launch_bounds__(256) void spec_tree_size_set(const TreeDesc *Dp, const TreeBufs *Bp, "
         "TableSet s) {\n"
      << "  const TreeDesc &D = *Dp;\n  const TreeBufs &B = *Bp;\n  bool err = false;\n"
      << "  const uint32_t x = s.t[blockIdx.y];\n  const uint64_t rows = B.rows[x];\n"
      << "  switch (x) {\n";
    for (uint32_t t = 0; t < D.ntables; t++) {
        const TTable &X = D.t[t];
        if (X.shape == spec::SHAPE_MESSAGE) {
            o << "  case " << t << ": for (uint64_t row = grid_first(); row < rows; row += grid_stride()) gen_srow_" << t
              << "(D, B, x, row, err); break;\n";
            continue;
        }
        // list elements: scalars, strings, bytes and structs with constant kinds (value_size /
        // struct_size's rules); other elements (any) by the run-time rule below
        const TField &F = D.f[X.field];
        const bool val = X.shape == spec::SHAPE_VALUE && F.elem >= spec::K_BOOL && F.elem <= spec::K_BYTES;
        if (!val && X.shape != spec::SHAPE_STRUCT) continue;
        o << "  case " << t << ":\n    for (uint64_t row = grid_first(); row < rows; row += grid_stride()) {\n";
        if (val) {
            o << "      uint64_t a[4];\n      load_value_k<" << (int)F.elem << ">(" << col_expr(F.col) << ", row, a);\n"
              << "      const uint64_t total = " << value_size_expr(F.elem, "a") << ";\n";
            if (F.elem == spec::K_STRING || F.elem == spec::K_BYTES)
                o << "      { const uint32_t off = (uint32_t)a[0], len = (uint32_t)(a[0] >> 32);\n"
                  << "        if ((uint64_t)len > MAX_SIZE || (uint64_t)off + len > B.heap_lens[" << F.col << "]) err = true; }\n";
        } else {
            for (uint32_t i = X.field + 1u; i < F.send; i++)
                if (D.f[i].kind != spec::K_STRUCT)
                    o << "      uint64_t m" << i << "[4];\n      load_value_k<" << (int)D.f[i].kind << ">(" << col_expr(D.f[i].col)
                      << ", row, m" << i << ");\n";
            gen_struct_size(o, D, X.field, "total", "      ");
        }
        o << "      if (total > 0xffffffffull) err = true;\n      B.size[x][row] = (uint32_t)total;\n    }\n    break;\n";
    }
    o << "  default:\n"
      << "    for (uint64_t row = grid_first(); row < rows; row += grid_stride()) {\n"
      << "      const uint64_t total = size_row_shaped(D, B, x, row, err);\n"
      << "      if (total > 0xffffffffull) err = true;\n"
      << "      B.size[x][row] = (uint32_t)total;\n"
      << "    }\n  }\n  if (err) *B.err = 1;\n}\n";
    // the level-fused writer: where the record-tile writer does not apply (or is switched off)
    if (!tree_tile(D)) {
        o << "extern \"C\" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void spec_tree_write_set("
             "const TreeDesc *Dp, const TreeBufs *Bp, TableSet s) {\n"
          << "  const TreeDesc &D = *Dp;\n  const TreeBufs &B = *Bp;\n"
          << "  if (!B.out || *B.err || *B.total > B.out_cap) return;\n"
          << "  const uint32_t x = s.t[blockIdx.y];\n  const uint64_t rows = B.rows[x];\n"
          << "  switch (x) {\n";
        for (uint32_t t = 0; t < D.ntables; t++)
            if (D.t[t].shape == spec::SHAPE_MESSAGE)
                o << "  case " << t << ":\n"
                  << "    for (uint64_t row = grid_first(); row < rows; row += grid_stride()) {\n"
                  // a row outside its owners' BEGIN ranges is not written, and neither is anything
                  // under it: its children's positions are marked unplaced (they may hold stale
                  // workspace bytes otherwise, and the next depth's writer would emit at them)
                  << (D.t[t].rel == spec::REL_MANY
                          ? "      if (!list_row_covered(D, B, x, row)) { gen_unplace_" + std::to_string(t) +
                                "(D, B, row); continue; }\n"
                          : std::string())
                  << "      const uint64_t start = x == 0 ? B.offsets[row] : B.pos[x][row];\n"
                  << "      if (start == ~0ull) { gen_unplace_" << t << "(D, B, row); continue; }\n"
                  << "      if (x == 0 && B.ends_out) B.ends_out[row] = start + B.size[0][row];\n"
                  // the records' rows are long: 16-byte chunk stores (BEmit16); the shorter rows of
                  // the tables below them keep the dword emitter (measured on pkg1: records 170 ->
                  // 134 us with BEmit16, the depth-1 tables 159 -> 180 us)
                  << (t == 0 ? "      BEmit16 em{B.out, start, start};\n" : "      BEmit em{{B.out}, start, start};\n")
                  << "      gen_wrow_" << t << "(em, D, B, row, start);\n"
                  << "    }\n    break;\n";
        o << "  default:\n"
          << "    for (uint64_t row = grid_first(); row < rows; row += grid_stride()) write_row_shaped(D, B, x, row);\n"
          << "  }\n}\n";
    }
    for (uint32_t x = 0; x < D.ntables; x++) {
        const TTable &T = D.t[x];
        has[x] = false;
        if (T.groot != x || !tree_group_ok(D, x)) continue;
        has[x] = true;
        o << "template <class Src>\n__device__ __forceinline__ void gen_row_" << x
          << "(const Src &s, const TreeDesc &D, const TreeBufs &B, uint64_t row, long long lo, long long hi, bool panic, "
             "uint2 *gr) {\n";
        if (T.shape == spec::SHAPE_VALUE) {
            const TField &F = D.f[T.field];
            o << "  Val v; int n;\n"
              << "  const bool ok = decode_value_kn<" << (int)F.elem << ">(s, lo, hi, 0, v, n);\n"
              << "  if (" << col_expr(F.col) << ") store_value_k<" << (int)F.elem << ">(" << col_expr(F.col) << ", row, v);\n"
              << "  store_u8(" << col_expr(T.status_col) << ", row, panic ? ST_PANIC : (ok ? ST_OK : ST_INVALID_VALUE));\n";
        } else if (T.shape == spec::SHAPE_STRUCT) {
            o << "  uint32_t sst = ST_OK;\n";
            gen_struct(o, D, T.field, "lo", "hi", "  ");
            o << "  store_u8(" << col_expr(T.status_col) << ", row, panic ? (uint32_t)ST_PANIC : sst);\n";
        } else {
            gen_message_table(o, D, x, "lo", "hi", true);
            gen_sub_tables(o, D, x, -1, nullptr, "tree_message_fallback");
        }
        o << "}\n"
          << "extern \"C\" __global__ __launch_bounds__(256) void spec_tree_group_" << x
          << "(const TreeDesc *Dp, const TreeBufs *Bp, uint32_t x, uint32_t slab, uint32_t wave_bytes, uint32_t rpw) {\n"
          << "  const TreeDesc &D = *Dp;\n"
          << "  const TreeBufs &B = *Bp;\n"
          << "  const uint64_t rows = dec_rows(D, B, x);\n"
          << "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
          << "  uint2 *gr = (uint2 *)(smem + (threadIdx.x >> 6) * wave_bytes + slab) + (threadIdx.x & 63);\n"
          << "  tree_rows(B, x, rows, slab, wave_bytes, rpw,\n"
          << "            [&](const TreeLds &s, uint64_t row, long long lo, long long hi, bool panic) {\n"
          << "              gen_row_" << x << "(s, D, B, row, lo, hi, panic, gr);\n"
          << "            },\n"
          << "            [&](const GlobalSrc &s, uint64_t row, long long lo, long long hi, bool panic) {\n"
          << "              gen_row_" << x << "(s, D, B, row, lo, hi, panic, gr);\n"
          << "            });\n"
          << "}\n"
          << "extern \"C\" __global__ __launch_bounds__(256) void spec_tree_group_" << x
          << "g(const TreeDesc *Dp, const TreeBufs *Bp, uint32_t x, uint32_t slab, uint32_t wave_bytes, uint32_t rpw) {\n"
          << "  const TreeDesc &D = *Dp;\n"
          << "  const TreeBufs &B = *Bp;\n"
          << "  const uint64_t rows = dec_rows(D, B, x);\n"
          << "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
          << "  uint2 *gr = (uint2 *)(smem + (threadIdx.x >> 6) * wave_bytes + slab) + (threadIdx.x & 63);\n"
          << "  tree_rows_global(B, x, rows, [&](const GlobalSrc &s, uint64_t row, long long lo, long long hi, bool panic) {\n"
          << "    gen_row_" << x << "(s, D, B, row, lo, hi, panic, gr);\n"
          << "  });\n"
          << "}\n";
        // (4 waves per 64 rows: 110 vs 100 us for pkg1 — registers cap it at 3 waves per SIMD,
        // so 3 slabs per CU instead of 4)
        if (x == 0) gen_pair_rows(o, D, x, 2);
    }
    // level-fused list groups: the groups one decode level holds (lists owned by the previous
    // level's groups, rows from HBM) in ONE launch, blockIdx.y picking the group — each group is
    // a chain of dependent loads per row, so side by side their latencies overlap
    // (one launch for all of them: split by register budget — lists of values / structs at ~40
    // VGPRs, lists of messages at ~120 — the two launches ran back to back, 75.5 vs 70.5 us for
    // pkg1; amdgpu_waves_per_eu 6 or 8 spills: 86-87 us)
    {
        o << "extern \"C\" __global__ __launch_bounds__(256) void spec_tree_group_set"
          << "(const TreeDesc *Dp, const TreeBufs *Bp, TableSet ts, uint32_t wave_bytes) {\n"
          << "  const TreeDesc &D = *Dp;\n  const TreeBufs &B = *Bp;\n"
          << "  const uint32_t x = ts.t[blockIdx.y];\n  const uint64_t rows = dec_rows(D, B, x);\n"
          << "  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];\n"
          << "  uint2 *gr = (uint2 *)(smem + (threadIdx.x >> 6) * wave_bytes) + (threadIdx.x & 63);\n"
          << "  switch (x) {\n";
        for (uint32_t x = 1; x < D.ntables; x++)
            if (has[x])
                o << "  case " << x << ":\n"
                  << "    tree_rows_global(B, x, rows, [&](const GlobalSrc &s, uint64_t row, long long lo, long long hi, "
                     "bool panic) {\n"
                  << "      gen_row_" << x << "(s, D, B, row, lo, hi, panic, gr);\n"
                  << "    });\n    break;\n";
        o << "  default: break;\n  }\n}\n";
    }
    if (tree_tile(D)) gen_tile(o, D);
    return o.str();
}

struct TreeEntry {
    hipModule_t mod = nullptr;
    // [x]: decode, staged rows; [TREE_MAX_T + x]: decode, rows from HBM; [2 TREE_MAX_T + x]:
    // decode on 2 waves per 64 rows (the root group, gen_pair_rows; nullptr if not split);
    // [4 TREE_MAX_T], [+1]: the
    // level-fused encode size / write kernels; [+2]: the level-fused list-group decode kernel;
    // [+3]: the record-tile writer (nullptr where gen_tile does not apply)
    hipFunction_t fn[4 * spec::TREE_MAX_T + 4] = {};
    bool failed = false;
};
std::unordered_map<std::string, TreeEntry> g_tree_cache;

} // namespace

namespace spec {

void jit_set_enabled(int on) { g_enabled = on ? 1 : 0; }

long long jit_compile_only_tree(const TreeDesc &D) {
    bool has[TREE_MAX_T];
    const std::string src = generate_tree(D, has);
    return (long long)compile_source(src, TREE).size();
}

// The schema-specialised group kernels of a tree: fn[x] for each group root x that has one
// (nullptr where the run-time kernel runs), fn[TREE_MAX_T + x] its variant without staging,
// fn[2 TREE_MAX_T + x] its 2-wave variant (root group only; nullptr when not split),
// fn[4 TREE_MAX_T] / fn[4 TREE_MAX_T + 1] the level-fused size / write kernels of the encoder,
// fn[4 TREE_MAX_T + 2] the level-fused list-group decode kernel, fn[4 TREE_MAX_T + 3] the
// record-tile writer (one of the two writers is generated: nullptr for the other); nullptr
// when the JIT is off or failed.
const hipFunction_t *jit_tree_kernels(const TreeDesc &D) {
    if (!enabled()) return nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    // a repeated tree is found by its descriptor's bytes, without regenerating the source (every
    // spec_encode_tree call looks its kernels up)
    struct Known {
        int dev;
        TreeDesc desc;
        const hipFunction_t *fn;
    };
    static std::vector<Known *> known;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (const Known *k : known)
            if (k->dev == dev && memcmp(&k->desc, &D, sizeof(TreeDesc)) == 0) return k->fn;
    }
    bool has[TREE_MAX_T];
    const std::string src = generate_tree(D, has);
    const std::string key = "tree:" + std::to_string(dev) + ":" + src;
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_tree_cache.find(key);
    if (it == g_tree_cache.end()) {
        TreeEntry e;
        const std::vector<char> code = compile_source(src, TREE);
        bool ok = !code.empty() && hipModuleLoadData(&e.mod, code.data()) == hipSuccess;
        if (ok)
            ok = hipModuleGetFunction(&e.fn[4 * TREE_MAX_T], e.mod, "spec_tree_size_set") == hipSuccess &&
                 hipModuleGetFunction(&e.fn[4 * TREE_MAX_T + 2], e.mod, "spec_tree_group_set") == hipSuccess &&
                 hipModuleGetFunction(&e.fn[4 * TREE_MAX_T + (tree_tile(D) ? 3 : 1)], e.mod,
                                      tree_tile(D) ? "spec_tree_write_tile" : "spec_tree_write_set") == hipSuccess;
        for (uint32_t x = 0; ok && x < D.ntables; x++) {
            if (!has[x]) continue;
            const std::string name = "spec_tree_group_" + std::to_string(x);
            ok = hipModuleGetFunction(&e.fn[x], e.mod, name.c_str()) == hipSuccess &&
                 hipModuleGetFunction(&e.fn[TREE_MAX_T + x], e.mod, (name + "g").c_str()) == hipSuccess;
            std::vector<char> sel[4];
            uint32_t tw[TREE_MAX_T];
            if (ok && x == 0 && pair_split(D, x, 2, sel, tw))
                ok = hipModuleGetFunction(&e.fn[2 * TREE_MAX_T + x], e.mod, (name + "p2").c_str()) == hipSuccess;
        }
        if (!ok) {
            (void)hipGetLastError();
            e.failed = true;
            fprintf(stderr, "spec_amd jit: tree compile/load failed, run-time tree kernels in use\n");
        }
        it = g_tree_cache.emplace(key, e).first;
    }
    const hipFunction_t *fn = it->second.failed ? nullptr : it->second.fn;
    Known *k = new Known;
    k->dev = dev;
    memcpy(&k->desc, &D, sizeof(TreeDesc));
    k->fn = fn;
    known.push_back(k);
    return fn;
}

long long jit_compile_only(const spec_schema *schema, double) {
    if (!has_flat_fast_path(schema)) return 0;
    return (long long)compile_code(schema, DECODE).size();
}

long long jit_compile_only_encode(const spec_schema *schema) {
    if (!has_encoder(schema)) return 0;
    return (long long)compile_code(schema, ENCODE).size();
}

int jit_prepare_decode_flat(const spec_schema *schema, double) { return lookup(schema, DECODE) ? 1 : 0; }

int jit_launch_decode_flat(const spec_schema *schema, const DecodeArgs &a, double avg_record, hipStream_t stream) {
    if (decode_slab_bytes(avg_record) == 0) return 0; // records too large for LDS: generic kernel
    const Entry *ent = lookup(schema, DECODE);
    if (!ent) return 0;
    hipFunction_t fn = ent->fn[a.f.errmask ? 1 : 0]; // the errmask variant for spec_decode_flat_errors
    if (a.n <= a.r0) return 1;
    const bool wide = schema->nfields > (uint32_t)FAST_MAX_FIELDS || [&] {
        for (uint32_t f = 0; f < schema->nfields; f++)
            if (schema->fields[f].tag > 255) return true;
        return false;
    }();
    if (flat_pair() >= (wide ? 1 : 2) && ent->fn[a.f.errmask ? 3 : 2] && !persistent_decode()) {
        // a wave pair per 64 records, one slab per pair (+ 256 B exchange, + 512 B of masks)
        DecodeArgs args = a;
        args.slab = decode_slab_bytes(avg_record);
        args.xcd = xcd_swizzle_decode();
        uint64_t groups = (a.n - a.r0 + 63) / 64;
        if (args.xcd) groups = (groups + 7) / 8 * 8;
        size_t size = sizeof(args);
        void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size,
                         HIP_LAUNCH_PARAM_END};
        hipError_t e = hipModuleLaunchKernel(ent->fn[a.f.errmask ? 3 : 2], (unsigned)groups, 1, 1,
                                             64 * SPEC_AB_FLAT_WAVES, 1, 1,
                                             args.slab + (SPEC_AB_FLAT_WAVES - 1) * (a.f.errmask ? 768 : 256), stream,
                                             nullptr, extra);
        return e == hipSuccess ? 1 : -1;
    }
    const DecodeLaunch L = decode_launch(a.n - a.r0, avg_record, device_cus(), persistent_decode(), decode_wpb());
    DecodeArgs args = a;
    args.slab = L.slab;
    args.xcd = xcd_swizzle_decode() && !persistent_decode();
    size_t size = sizeof(args);
    void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size,
                     HIP_LAUNCH_PARAM_END};
    hipError_t e = hipModuleLaunchKernel(fn, L.blocks, 1, 1, 64 * L.wpb, 1, 1, L.lds, stream, nullptr, extra);
    return e == hipSuccess ? 1 : -1;
}

int jit_launch_encode(const spec_schema *schema, const EncodeArgs &a, bool write, hipStream_t stream) {
    const Entry *e = lookup(schema, ENCODE);
    if (!e) return 0;
    EncodeArgs args = a;
    size_t size = sizeof(args);
    void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size,
                     HIP_LAUNCH_PARAM_END};
    hipError_t rc;
    if (write && e->fn[2]) { // the write pass on wave pairs (encode_write_pair_body)
        const int h = enc_pair_split(schema);
        rc = hipModuleLaunchKernel(e->fn[2], (unsigned)a.nblocks, 1, 1, ENC_PAIR_BLOCK, 1, 1,
                                   (unsigned)enc_pair_lds_bytes(h), stream, nullptr, extra);
    } else {
        rc = hipModuleLaunchKernel(e->fn[write ? 1 : 0], (unsigned)a.nblocks, 1, 1, ENC_BLOCK, 1, 1,
                                   write ? (unsigned)enc_write_lds_bytes() : 0, stream, nullptr, extra);
    }
    return rc == hipSuccess ? 1 : -1;
}

long long jit_compile_only_nested(const spec_nested_schema *schema) {
    if (!has_nested_fast_path(schema)) return 0;
    return (long long)compile_source(generate_nested(schema), NESTED).size();
}

int jit_launch_nested(const spec_nested_schema *schema, const NestedArgs &a, int mode, hipStream_t stream) {
    if (a.slab == 0) return 0; // records too large for LDS: generic kernel
    const Entry *e = lookup_nested(schema);
    if (!e) return 0;
    NestedArgs args = a;
    size_t size = sizeof(args);
    void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size,
                     HIP_LAUNCH_PARAM_END};
    unsigned grid = (unsigned)((a.n + 63) / 64);
    if (args.xcd && mode != NESTED_ONEPASS) grid = (grid + 7) / 8 * 8; // 8 equal XCD shares
    else args.xcd = 0;
    size_t lds = a.slab + (mode == NESTED_RANGES ? NESTED_RANGE_BYTES : 0u);
    unsigned threads = 64;
    if (mode == NESTED_GROUPS && nested_pair() && e->fn[3]) { // a wave pair per group (nested_decode_pair)
        mode = 3;
        threads = 64 * SPEC_AB_NESTED_WAVES;
        lds = a.slab + 1024; // the posted lists: 4 words per record
    }
    if (mode == NESTED_PAIR_ONEPASS) { // a wave pair per group, one look-back per group, block order
        if (!e->fn[4]) return 0;
        args.xcd = 0;
        hipError_t rc = hipModuleLaunchKernel(e->fn[4], (unsigned)((a.n + 63) / 64), 1, 1, 64 * SPEC_AB_NESTED_WAVES, 1,
                                              1, a.slab + 1024 + 16, stream, nullptr, extra);
        return rc == hipSuccess ? 1 : -1;
    }
    if (mode == NESTED_ONEPASS) { // DEC_WAVES groups per block: one look-back per block
        grid = (grid + DEC_WAVES - 1) / DEC_WAVES;
        threads = 64 * DEC_WAVES;
        lds *= DEC_WAVES;
    }
    hipError_t rc = hipModuleLaunchKernel(e->fn[mode], grid, 1, 1, threads, 1, 1, (unsigned)lds, stream, nullptr, extra);
    return rc == hipSuccess ? 1 : -1;
}

long long jit_compile_only_nested_encode(const spec_nested_schema *schema) {
    if (!has_nested_encoder(schema)) return 0;
    return (long long)compile_source(generate_nested_encode(schema), NESTED_ENC).size();
}

#ifndef SPEC_AB_NENC_PAIR
#define SPEC_AB_NENC_PAIR 1
#endif
int jit_launch_nested_encode(const spec_nested_schema *schema, const NestedEncodeArgs &a, bool write,
                             hipStream_t stream) {
    const Entry *e = lookup_nested_encode(schema);
    if (!e) return 0;
    NestedEncodeArgs args = a;
    args.xcd = write && xcd_swizzle_decode() ? 1u : 0u;
    size_t size = sizeof(args);
    void *extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &args, HIP_LAUNCH_PARAM_BUFFER_SIZE, &size,
                     HIP_LAUNCH_PARAM_END};
    const unsigned lds = (unsigned)(write ? nenc_write_lds_bytes() : nenc_size_lds_bytes());
    const unsigned grid = (unsigned)(args.xcd ? (a.nblocks + 7) / 8 * 8 : a.nblocks);
    // the write pass on wave pairs when the size pass left its item prefixes (nested_enc_write_pair_body)
    const bool pair = write && SPEC_AB_NENC_PAIR && e->fn[2] && a.item_pre && a.wave_ok;
    hipError_t rc = hipModuleLaunchKernel(e->fn[pair ? 2 : write ? 1 : 0], grid, 1, 1, pair ? 2 * NENC_BLOCK : NENC_BLOCK,
                                          1, 1, lds, stream, nullptr, extra);
    return rc == hipSuccess ? 1 : -1;
}

} // namespace spec

// capi.cpp -- C entry point of the host CLI for bindings and tests
// (ctypes in kafkabalancer_amd/cli.py): kb_cli_run mirrors run(i, o, e, args).
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <chrono>

#include "cli.hpp"
#include "codecs.hpp"

extern "C" int kb_cli_run(int argc, const char* const* argv, const char* stdin_data, size_t stdin_len,
                          int fail_output, char** out, size_t* out_len, char** err, size_t* err_len) {
    std::vector<std::string> args;
    for (int i = 0; i < argc; i++) args.emplace_back(argv[i]);
    std::string o, e;
    int rc = kbh::Run(args, [&](bool* ok) {
        *ok = stdin_data != nullptr;
        return stdin_data ? std::string(stdin_data, stdin_len) : std::string();
    }, &o, &e, fail_output != 0);
    *out = (char*)malloc(o.size() + 1);
    memcpy(*out, o.data(), o.size());
    (*out)[o.size()] = 0;
    *out_len = o.size();
    *err = (char*)malloc(e.size() + 1);
    memcpy(*err, e.data(), e.size());
    (*err)[e.size()] = 0;
    *err_len = e.size();
    return rc;
}

extern "C" void kb_cli_free(void* p) { free(p); }

// Codec entry for the throughput bench and the fast-path parity tests: decode `in`
// (JSON, codecs.go:15-27) and encode the result (codecs.go:84-93).  mode 0: the
// CLI's path (one-pass decoder, DOM fallback), 1: DOM parser + decoder only, 2: the
// one-pass decoder only (returns 2 when it gives up).  Returns 0 with the encoded
// bytes in *out, or 1 with the error text in *out; t_parse / t_encode in seconds.
extern "C" int kb_codec_roundtrip(const char* in, size_t len, int mode, char** out, size_t* out_len,
                                  double* t_parse, double* t_encode, int64_t* n_parts) {
    const std::string src(in, len);
    kbh::PartitionList pl;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    std::string err;
    if (mode == 2) {
        if (!kbh::FastDecodePartitionList(src, &pl)) return 2;
    } else {
        const bool save = kbh::g_codec_dom_only;
        kbh::g_codec_dom_only = mode == 1;
        err = kbh::GetPartitionListFromReader(src, true, {}, &pl);
        kbh::g_codec_dom_only = save;
    }
    const auto t1 = clk::now();
    std::string o = err.empty() ? kbh::EncodePartitionList(pl) : err;
    const auto t2 = clk::now();
    *t_parse = std::chrono::duration<double>(t1 - t0).count();
    *t_encode = err.empty() ? std::chrono::duration<double>(t2 - t1).count() : 0.0;
    *n_parts = (int64_t)pl.partitions.size();
    *out = (char*)malloc(o.size() + 1);
    memcpy(*out, o.data(), o.size());
    (*out)[o.size()] = 0;
    *out_len = o.size();
    return err.empty() ? 0 : 1;
}

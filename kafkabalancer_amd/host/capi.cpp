// capi.cpp -- C entry point of the host CLI for bindings and tests
// (ctypes in kafkabalancer_amd/cli.py): kb_cli_run mirrors run(i, o, e, args).
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cli.hpp"

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

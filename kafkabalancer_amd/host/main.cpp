// main.cpp -- the kafkabalancer executable (kafkabalancer.go:68-70).
#include <cstdio>
#include <iostream>
#include <iterator>
#include <string>
#include <vector>

#include "cli.hpp"

int main(int argc, char** argv) {
    std::vector<std::string> args(argv, argv + argc);
    if (!args.empty()) args[0] = "kafkabalancer";
    std::string out, err;
    int rc = kbh::Run(args, [](bool* ok) {
        std::string s((std::istreambuf_iterator<char>(std::cin)), std::istreambuf_iterator<char>());
        *ok = !std::cin.bad();
        return s;
    }, &out, &err);
    fwrite(err.data(), 1, err.size(), stderr);
    if (!out.empty()) {
        size_t w = fwrite(out.data(), 1, out.size(), stdout);
        if (fflush(stdout) != 0 || w != out.size()) {
            fprintf(stderr, "failed writing partition list: failed serializing json: write error\n");
            return 4;
        }
    }
    return rc;
}

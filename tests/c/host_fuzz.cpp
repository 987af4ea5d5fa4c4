// host_fuzz.cpp -- the native host side (kafkabalancer_amd/host: codecs, CLI) driven
// by mutated inputs, built with -fsanitize=address,undefined by
// tests/test_host_sanitizers.py (host code only; no GPU is touched: every CLI run
// below ends before an engine would be created, or fails creating it).
//
// Checks, per mutated document:
//   * JSON (codecs.go:15-27): the CLI's decoder (one-pass, DOM fallback) and the DOM
//     decoder agree on the error text or on the encoded bytes (codecs.go:84-93);
//   * text (`kafka-topics.sh --describe`, codecs.go:28-56): decoding terminates and
//     an accepted list encodes;
//   * the CLI (kafkabalancer.go:72-242) on mutated argument vectors and inputs.
// Usage: host_fuzz SEED_JSON SEED_TEXT ITERATIONS
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../kafkabalancer_amd/host/cli.hpp"
#include "../../kafkabalancer_amd/host/codecs.hpp"

namespace {

uint64_t g_rng = 0x9E3779B97F4A7C15ull;
uint64_t next() {   // splitmix64
    uint64_t z = (g_rng += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
size_t below(size_t n) { return n ? (size_t)(next() % n) : 0; }

std::string slurp(const char* path) {
    std::ifstream f(path, std::ios::binary);
    std::stringstream s;
    s << f.rdbuf();
    return s.str();
}

std::string mutate(const std::string& base, const std::string& alphabet) {
    std::string b = base;
    const int n = 1 + (int)below(4);
    for (int i = 0; i < n; i++) {
        const size_t k = below(b.size() + 1);
        switch (below(5)) {
            case 0: if (k < b.size()) b.erase(k, 1); break;
            case 1: b.insert(b.begin() + (long)k, alphabet[below(alphabet.size())]); break;
            case 2: if (k < b.size()) b[k] = alphabet[below(alphabet.size())]; break;
            case 3: b = b.substr(0, k); break;                                   // truncation
            default: {                                                           // splice a chunk
                const size_t a = below(b.size() + 1), len = below(64);
                b.insert(k, b.substr(a, len));
            }
        }
    }
    return b;
}

int fails = 0;

void check_json(const std::string& doc) {
    kbh::PartitionList a, b;
    kbh::g_codec_dom_only = false;
    const std::string ea = kbh::GetPartitionListFromReader(doc, true, {}, &a);
    kbh::g_codec_dom_only = true;
    const std::string eb = kbh::GetPartitionListFromReader(doc, true, {}, &b);
    kbh::g_codec_dom_only = false;
    if (ea != eb) {
        if (fails++ < 5) fprintf(stderr, "decode mismatch: '%s' vs '%s'\n", ea.c_str(), eb.c_str());
        return;
    }
    if (ea.empty() && kbh::EncodePartitionList(a) != kbh::EncodePartitionList(b)) {
        if (fails++ < 5) fprintf(stderr, "encode mismatch\n");
    }
    kbh::PartitionList c;
    (void)kbh::FastDecodePartitionList(doc, &c);
    (void)kbh::FilterPartitionList(a);
}

void check_text(const std::string& doc, const std::vector<std::string>& topics) {
    kbh::PartitionList pl;
    if (kbh::GetPartitionListFromReader(doc, false, topics, &pl).empty()) (void)kbh::EncodePartitionList(pl);
}

void check_cli(const std::string& doc) {
    static const char* flags[] = {"-input-json", "-max-reassign", "-allow-leader", "-broker-ids", "-min-unbalance",
                                  "-topics", "-full-output", "-unique", "-complete-partition", "-min-replicas",
                                  "-rebalance-leader", "-input", "-help", "-h", "--", "-x"};
    static const char* vals[] = {"0", "-1", "1,2,x", "", "1e9", "abc", "true", "=false", "3", "0.5", "nan", "/nonexistent"};
    std::vector<std::string> args{"kafkabalancer"};
    const int n = (int)below(5);
    for (int i = 0; i < n; i++) {
        std::string f = flags[below(sizeof flags / sizeof *flags)];
        if (below(2)) f += std::string("=") + vals[below(sizeof vals / sizeof *vals)];
        args.push_back(f);
        if (below(3) == 0) args.push_back(vals[below(sizeof vals / sizeof *vals)]);
    }
    // -max-reassign 0 keeps a run that parses to the end away from the engine
    args.push_back("-max-reassign=0");
    std::string out, err;
    (void)kbh::Run(args, [&](bool* ok) { *ok = true; return doc; }, &out, &err, below(8) == 0);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage: host_fuzz SEED_JSON SEED_TEXT ITERATIONS\n"); return 2; }
    const std::string js = slurp(argv[1]), tx = slurp(argv[2]);
    const long iters = atol(argv[3]);
    const std::string ja = "{}[]:,\"-.0123456789eEnultrfas \\\tx\xc3\xa9";
    const std::string ta = "\t\n:, 0123456789TopicPartitionLeaderReplicasIsr-x";
    check_json(js);
    check_text(tx, {});
    for (long i = 0; i < iters; i++) {
        check_json(mutate(js, ja));
        check_text(mutate(tx, ta), below(2) ? std::vector<std::string>{} : std::vector<std::string>{"t00000", "x"});
        if (i % 4 == 0) check_cli(below(2) ? mutate(js, ja) : mutate(tx, ta));
    }
    if (fails) { fprintf(stderr, "%d mismatches\n", fails); return 1; }
    printf("host-fuzz-ok %ld\n", iters);
    return 0;
}

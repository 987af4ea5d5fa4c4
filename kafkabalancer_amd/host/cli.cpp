// cli.cpp -- the kafkabalancer command line (kafkabalancer.go:68-242) on the
// MI355X engine: same flags, defaults, log lines and exit codes
// (0 ok, 1 input file, 2 parse, 3 config/balance, 4 output).
//
// Extensions (not in the reference): -semantics=go|applied (default go: Go
// slice aliasing) and -device N.  -from-zk (ZooKeeper ingest) is
// out of scope: it fails like an unreachable ZooKeeper (exit 2).
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "balancer.hpp"
#include "codecs.hpp"
#include "cli.hpp"

namespace kbh {

namespace {

struct Log {
    std::string* sink;
    void print(const std::string& m) {                    // log.Printf with LstdFlags
        char ts[32];
        time_t t = time(nullptr);
        struct tm tmv;
        localtime_r(&t, &tmv);
        strftime(ts, sizeof ts, "%Y/%m/%d %H:%M:%S ", &tmv);
        *sink += ts;
        *sink += m;
        if (m.empty() || m.back() != '\n') *sink += '\n';
    }
};

struct FlagDef {
    std::string name, type, usage, defval;   // type: "bool", "string", "int", "float"
    std::string value;
    bool is_bool() const { return type == "bool"; }
};

bool parse_bool(const std::string& s, bool* v) {          // strconv.ParseBool
    static const char* t[] = {"1", "t", "T", "TRUE", "true", "True"};
    static const char* f[] = {"0", "f", "F", "FALSE", "false", "False"};
    for (auto x : t) if (s == x) { *v = true; return true; }
    for (auto x : f) if (s == x) { *v = false; return true; }
    return false;
}

bool parse_int(const std::string& s, int64_t* v) {        // strconv.ParseInt(s, 0, 64)
    if (s.empty()) return false;
    std::string t = s;
    bool neg = false;
    size_t i = 0;
    if (t[0] == '+' || t[0] == '-') { neg = t[0] == '-'; i = 1; }
    int base = 10;
    if (t.size() > i + 1 && t[i] == '0' && (t[i + 1] == 'x' || t[i + 1] == 'X')) { base = 16; i += 2; }
    else if (t.size() > i + 1 && t[i] == '0' && (t[i + 1] == 'b' || t[i + 1] == 'B')) { base = 2; i += 2; }
    else if (t.size() > i + 1 && t[i] == '0' && (t[i + 1] == 'o' || t[i + 1] == 'O')) { base = 8; i += 2; }
    else if (t.size() > i + 1 && t[i] == '0') { base = 8; i += 1; }
    std::string digits;
    for (; i < t.size(); i++) if (t[i] != '_') digits += t[i];
    if (digits.empty()) return false;
    errno = 0;
    char* end = nullptr;
    unsigned long long u = strtoull(digits.c_str(), &end, base);
    if (errno || *end) return false;
    if (!neg && u > 9223372036854775807ull) return false;
    if (neg && u > 9223372036854775808ull) return false;
    *v = neg ? (int64_t)(0 - u) : (int64_t)u;
    return true;
}

bool parse_float(const std::string& s, double* v) {       // strconv.ParseFloat(s, 64)
    if (s.empty()) return false;
    errno = 0;
    char* end = nullptr;
    double x = strtod(s.c_str(), &end);
    if (*end) return false;
    if (errno == ERANGE && std::isinf(x)) return false;
    *v = x;
    return true;
}

// strconv.Atoi for -broker-ids elements (base 10, optional sign)
bool atoi_strict(const std::string& s, int64_t* v, std::string* err) {
    bool ok = !s.empty();
    size_t i = (s.size() && (s[0] == '+' || s[0] == '-')) ? 1 : 0;
    if (i == s.size()) ok = false;
    for (size_t k = i; ok && k < s.size(); k++) ok = isdigit((unsigned char)s[k]);
    if (ok) {
        errno = 0;
        long long x = strtoll(s.c_str(), nullptr, 10);
        if (errno == ERANGE) { *err = "strconv.Atoi: parsing \"" + s + "\": value out of range"; return false; }
        *v = x;
        return true;
    }
    *err = "strconv.Atoi: parsing \"" + s + "\": invalid syntax";
    return false;
}

std::string go_quote(const std::string& s) { return "\"" + s + "\""; }

}  // namespace

int Run(const std::vector<std::string>& args, const std::function<std::string(bool*)>& read_stdin,
        std::string* out, std::string* err, bool fail_output) {
    Log log{err};
    std::vector<FlagDef> flags = {
        {"input-json", "bool", "Parse the input as JSON", "false", "false"},
        {"input", "string", "Name of the file to read (if no file is specified read from stdin, can not be used with -from-zk)", "", ""},
        {"from-zk", "string", "Zookeeper connection string (can not be used with -input)", "", ""},
        {"max-reassign", "int", "Maximum number of reassignments to generate", "1", "1"},
        {"full-output", "bool", "Output the full partition list: by default only the changes are printed", "false", "false"},
        {"unique", "bool", "Output only unique topic+partition", "false", "false"},
        {"pprof", "bool", "Enable CPU profiling", "false", "false"},
        {"allow-leader", "bool", "Consider the partition leader eligible for rebalancing", "false", "false"},
        {"rebalance-leader", "bool", "Force rebalance leadership", "false", "false"},
        {"complete-partition", "bool", "Force to always complete a topic+partition's replicas to be valid.", "true", "true"},
        {"topics", "string", "Only process these commaseparated topics", "", ""},
        {"min-replicas", "int", "Minimum number of replicas for a partition to be eligible for rebalancing", "2", "2"},
        {"min-unbalance", "float", "Minimum unbalance value required to perform rebalancing", "0.01", "0.01"},
        {"broker-ids", "string", "Comma-separated list of broker IDs", "auto", "auto"},
        {"help", "bool", "Display usage", "false", "false"},
        {"semantics", "string", "Plan semantics: go (reference slice aliasing) or applied (every change applied)", "go", "go"},
        {"device", "int", "HIP device ordinal", "0", "0"},
    };
    std::map<std::string, FlagDef*> byname;
    for (auto& f : flags) byname[f.name] = &f;
    const std::string prog = args.empty() ? "kafkabalancer" : args[0];
    auto usage = [&]() {                                   // f.Usage + PrintDefaults
        std::string u = "Usage of " + prog + ":\n";
        std::vector<FlagDef*> sorted;
        for (auto& f : flags) sorted.push_back(&f);
        std::sort(sorted.begin(), sorted.end(), [](FlagDef* a, FlagDef* b) { return a->name < b->name; });
        for (FlagDef* f : sorted) {
            std::string line = "  -" + f->name;
            std::string tn = f->type == "bool" ? "" : (f->type == "float" ? "float" : f->type);
            if (!tn.empty()) line += " " + tn;
            line += (line.size() <= 4) ? "\t" : "\n    \t";
            line += f->usage;
            bool zero = (f->type == "bool" && f->defval == "false") || (f->type == "string" && f->defval.empty()) ||
                        ((f->type == "int" || f->type == "float") && f->defval == "0");
            if (!zero) line += f->type == "string" ? " (default " + go_quote(f->defval) + ")" : " (default " + f->defval + ")";
            u += line + "\n";
        }
        *err += u;
    };

    // flag.Parse (ContinueOnError); the reference ignores the returned error
    // (kafkabalancer.go:98): parsing just stops at a bad flag
    for (size_t i = 1; i < args.size(); i++) {
        std::string a = args[i];
        if (a.size() < 2 || a[0] != '-') break;
        size_t dashes = (a[1] == '-') ? 2 : 1;
        if (dashes == 2 && a.size() == 2) break;               // "--" terminates
        std::string name = a.substr(dashes), val;
        bool has_val = false;
        if (name.empty() || name[0] == '-' || name[0] == '=') {
            *err += "bad flag syntax: " + a + "\n";
            usage();
            break;
        }
        size_t eq = name.find('=');
        if (eq != std::string::npos) { val = name.substr(eq + 1); name = name.substr(0, eq); has_val = true; }
        auto it = byname.find(name);
        if (it == byname.end()) {
            if (name == "h" || name == "help") { usage(); break; }
            *err += "flag provided but not defined: -" + name + "\n";
            usage();
            break;
        }
        FlagDef* f = it->second;
        if (f->is_bool()) {
            bool b = true;
            if (has_val && !parse_bool(val, &b)) {
                *err += "invalid boolean value " + go_quote(val) + " for -" + name + ": parse error\n";
                usage();
                break;
            }
            f->value = b ? "true" : "false";
        } else {
            if (!has_val) {
                if (i + 1 >= args.size()) { *err += "flag needs an argument: -" + name + "\n"; usage(); break; }
                val = args[++i];
            }
            if (f->type == "int") {
                int64_t x;
                if (!parse_int(val, &x)) { *err += "invalid value " + go_quote(val) + " for flag -" + name + ": parse error\n"; usage(); break; }
                f->value = std::to_string((long long)x);
            } else if (f->type == "float") {
                double x;
                if (!parse_float(val, &x)) { *err += "invalid value " + go_quote(val) + " for flag -" + name + ": parse error\n"; usage(); break; }
                f->value = val;
            } else {
                f->value = val;
            }
        }
    }
    auto B = [&](const char* n) { return byname[n]->value == "true"; };
    auto S = [&](const char* n) { return byname[n]->value; };
    auto I = [&](const char* n) { int64_t x = 0; parse_int(byname[n]->value, &x); return x; };

    if (B("help")) { usage(); return 0; }

    RebalanceConfig cfg;
    std::string bids = S("broker-ids");
    if (bids != "auto") {
        cfg.brokers_nil = false;
        size_t a = 0;
        for (;;) {
            size_t c = bids.find(',', a);
            std::string tok = bids.substr(a, c == std::string::npos ? std::string::npos : c - a);
            int64_t b;
            std::string e;
            if (!atoi_strict(tok, &b, &e)) {
                log.print("failed parsing broker list \"" + bids + "\": " + e);
                usage();
                return 3;
            }
            cfg.brokers.push_back(b);
            if (c == std::string::npos) break;
            a = c + 1;
        }
    }
    int64_t max_reassign = I("max-reassign");
    if (max_reassign < 0) {
        log.print("invalid number of max reassignments \"" + std::to_string((long long)max_reassign) + "\"");
        usage();
        return 3;
    }
    std::string input = S("input"), zk = S("from-zk");
    if (!input.empty() && !zk.empty()) {
        log.print("can't specify both -input and -from-zk");
        usage();
        return 3;
    }
    // diagnostic phase wall times (KB_CLI_TIMINGS=<file>: one JSON line appended; what a
    // drop-in user pays end to end, bench.py --drop-in)
    using clk = std::chrono::steady_clock;
    const clk::time_point t_start = clk::now();
    double t_read = 0, t_decode = 0, t_create = 0, t_plan = 0, t_encode = 0;
    auto secs = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); };
    std::string data;
    if (!input.empty()) {
        FILE* fp = fopen(input.c_str(), "rb");
        if (!fp) {
            std::string why = strerror(errno);                 // Go prints syscall errors in lower case
            if (!why.empty()) why[0] = (char)tolower((unsigned char)why[0]);
            log.print("failed opening file " + input + ": open " + input + ": " + why);
            return 1;
        }
        char buf[1 << 16];
        size_t k;
        while ((k = fread(buf, 1, sizeof buf, fp)) > 0) data.append(buf, k);
        fclose(fp);
    }
    std::vector<std::string> topics;
    {
        std::string t = S("topics");
        size_t a = 0;
        for (;;) {
            size_t c = t.find(',', a);
            std::string tok = t.substr(a, c == std::string::npos ? std::string::npos : c - a);
            if (!tok.empty()) topics.push_back(tok);
            if (c == std::string::npos) break;
            a = c + 1;
        }
    }
    PartitionList pl;
    std::string perr;
    clk::time_point t_mark = clk::now();
    t_read = secs(t_start, t_mark);
    if (!zk.empty()) {
        perr = "failed parsing zk connection string: ZooKeeper ingest is not supported by this build (" + zk + ")";
    } else {
        if (input.empty()) {
            bool ok = true;
            data = read_stdin(&ok);
            if (!ok) perr = "failed reading file: read error";
        }
        if (perr.empty()) perr = GetPartitionListFromReader(data, B("input-json"), topics, &pl);
    }
    if (!perr.empty()) {
        log.print("failed getting partition list: " + perr);
        return 2;
    }
    { const clk::time_point t = clk::now(); t_decode = secs(t_mark, t); t_mark = t; }

    cfg.allow_leader = B("allow-leader");
    cfg.rebalance_leaders = B("rebalance-leader");
    cfg.min_replicas = I("min-replicas");
    {
        double x = 0.01;
        parse_float(S("min-unbalance"), &x);
        cfg.min_unbalance = x;
    }
    cfg.complete_partition = B("complete-partition");
    std::string bl = "[";
    for (size_t k = 0; k < cfg.brokers.size(); k++) bl += (k ? " " : "") + std::to_string((long long)cfg.brokers[k]);
    bl += "]";
    // CompletePartition is not copied into cfg by the reference (kafkabalancer.go:167-173)
    log.print(std::string("rebalance config: {AllowLeaderRebalancing:") + (cfg.allow_leader ? "true" : "false") +
              " RebalanceLeaders:" + (cfg.rebalance_leaders ? "true" : "false") +
              " MinReplicasForRebalancing:" + std::to_string((long long)cfg.min_replicas) +
              " MinUnbalance:" + GoFloatG(cfg.min_unbalance) + " CompletePartition:false Brokers:" + bl + "}");
    const int sem = S("semantics") == "applied" ? KB_SEM_APPLIED : KB_SEM_GO;

    PartitionList opl;
    opl.version = 1;
    Planner planner(pl, cfg, sem, (int)I("device"));
    if (!planner.ok()) {
        log.print("failed optimizing distribution: " + planner.error());
        return 3;
    }
    { const clk::time_point t = clk::now(); t_create = secs(t_mark, t); t_mark = t; }
    bool completing = false;
    Partition cpart;
    int64_t r = max_reassign;
    int64_t iters = 0;
    const int64_t guard = max_reassign + 1000000;
    std::vector<StepResult> pending;
    // device-resident: the first -max-reassign changes in one plan (every mode: the completing
    // logic starts only after them), then the -complete-partition loop in batches that stop
    // after the first change on another partition (kb_engine_plan_until)
    if (r > 0) pending = planner.Plan(r);
    size_t pi = 0;
    int64_t cidx = -1;                                      // the completing partition's index
    while (r > 0) {                                         // MainLoop (kafkabalancer.go:181-221)
        if (pi >= pending.size() && completing) {
            pending = planner.PlanUntil(64, cidx);
            pi = 0;
        }
        StepResult sr = pi < pending.size() ? pending[pi++] : planner.Step();
        if (++iters > guard) {
            log.print("plan does not terminate: the reference loops forever on this input (-complete-partition)");
            return 5;
        }
        if (sr.status < 0) {
            if (sr.status == KB_ERR_PANIC) {
                *err += "panic: " + sr.err + "\n";
                return 2;
            }
            log.print("failed optimizing distribution: " + sr.err);
            return 3;
        }
        if (sr.status == KB_NOCHANGE) {
            log.print("no candidate changes");
            break;
        }
        log.print(sr.step + ": PartitionList([" + sr.part.str() + "])");
        if (!completing) {
            opl.partitions.push_back(sr.part);
            opl.nil_partitions = false;
        } else {
            if (cpart.same(sr.part)) {
                opl.partitions.push_back(sr.part);
            } else {
                log.print("Partition " + sr.part.str() + " did not compare.");
                break;
            }
        }
        r--;
        if (r == 0 && cfg.complete_partition) {
            r = 1;
            if (!completing) {
                cpart = opl.partitions.back();
                cidx = sr.change.partition;
                completing = true;
                log.print("Forcing complete of Partition: " + cpart.str());
            }
        }
    }
    { const clk::time_point t = clk::now(); t_plan = secs(t_mark, t); t_mark = t; }
    PartitionList* res = &opl;
    PartitionList filtered;
    if (B("full-output")) res = &pl;
    if (B("unique")) { filtered = FilterPartitionList(*res); res = &filtered; }
    log.print("Writing " + std::to_string(res->partitions.size()) + " changes.");
    std::string bytes = EncodePartitionList(*res);
    t_encode = secs(t_mark, clk::now());
    if (const char* tf = getenv("KB_CLI_TIMINGS")) {
        if (FILE* fp = fopen(tf, "a")) {
            fprintf(fp, "{\"read_s\": %.6f, \"decode_s\": %.6f, \"create_s\": %.6f, \"plan_s\": %.6f, "
                        "\"encode_s\": %.6f, \"input_bytes\": %zu, \"partitions\": %zu, \"changes\": %zu, "
                        "\"output_bytes\": %zu}\n",
                    t_read, t_decode, t_create, t_plan, t_encode, data.size(), pl.partitions.size(),
                    opl.partitions.size(), bytes.size());
            fclose(fp);
        }
    }
    if (fail_output) {
        log.print("failed writing partition list: failed serializing json: write failed");
        return 4;
    }
    *out += bytes;
    return 0;
}

}  // namespace kbh

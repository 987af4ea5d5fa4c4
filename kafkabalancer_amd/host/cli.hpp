// cli.hpp -- run() of the reference CLI (kafkabalancer.go:72-242).
#pragma once
#include <functional>
#include <string>
#include <vector>

namespace kbh {
// args[0] is the program name.  read_stdin is called only when the input comes
// from stdin.  fail_output emulates a failing writer (kafkabalancer_test.go:127-143).
int Run(const std::vector<std::string>& args, const std::function<std::string(bool*)>& read_stdin,
        std::string* out, std::string* err, bool fail_output = false);
}  // namespace kbh

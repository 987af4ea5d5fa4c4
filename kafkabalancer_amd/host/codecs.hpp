// codecs.hpp -- GetPartitionListFromReader / WritePartitionList /
// FilterPartitionList (codecs.go:15-93) with Go encoding/json behaviour.
#pragma once
#include <string>
#include <vector>

#include "model.hpp"

namespace kbh {

// codecs.go:15-64.  Returns "" on success or the reference's error text.
std::string GetPartitionListFromReader(const std::string& in, bool json,
                                       const std::vector<std::string>& topics, PartitionList* out);

// codecs.go:84-93: Go encoding/json bytes of pl (Version forced to 1) + "\n"
std::string EncodePartitionList(PartitionList& pl);

// the one-pass decoder alone (no DOM): true when it produced the PartitionList the
// DOM parser + decoder would, false when it gave up (unusual or invalid input)
bool FastDecodePartitionList(const std::string& in, PartitionList* out);
extern bool g_codec_dom_only;   // diagnostic / tests: always take the DOM path

// codecs.go:67-82
PartitionList FilterPartitionList(const PartitionList& pl);

// Go encoding/json float64 text (strconv 'f'/-1, 'e' outside [1e-6, 1e21))
std::string GoFloat(double x);
void GoFloatAppend(std::string& o, double x);

// fmt %v of a float64 (strconv 'g' shortest), used in log lines
std::string GoFloatG(double x);

}  // namespace kbh

// model.hpp -- the reference data model (kafkabalancer.go:16-66) on the host.
//
// Replicas/Brokers are Go slices: a shared backing array + a length, so the
// plan entries alias the partition list exactly like the reference's
// replacepl() results do (utils.go:166-197).
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace kbh {

struct Slice {
    std::shared_ptr<std::vector<int64_t>> arr;   // null => nil slice
    size_t len = 0;

    bool nil() const { return !arr; }
    int64_t at(size_t i) const { return (*arr)[i]; }
    int64_t& at(size_t i) { return (*arr)[i]; }
    std::vector<int64_t> values() const {
        if (!arr) return {};
        return std::vector<int64_t>(arr->begin(), arr->begin() + (long)len);
    }
    static Slice of(const std::vector<int64_t>& v) {
        Slice s;
        s.arr = std::make_shared<std::vector<int64_t>>(v);
        s.len = v.size();
        return s;
    }
    static Slice empty() { return of({}); }
};

struct Partition {
    std::string topic;          // TopicName
    int64_t partition = 0;      // PartitionID
    Slice replicas;             // []BrokerID
    double weight = 0;          // Weight
    int64_t num_replicas = 0;   // NumReplicas
    Slice brokers;              // Brokers (nil = default)
    int64_t num_consumers = 0;  // NumConsumers

    // Partition.String() (kafkabalancer.go:64-66)
    std::string str() const;
    bool same(const Partition& o) const { return topic == o.topic && partition == o.partition; }
};

struct PartitionList {
    int64_t version = 0;
    bool nil_partitions = true;
    std::vector<Partition> partitions;
};

struct RebalanceConfig {          // balancer.go:12-20
    bool allow_leader = false;
    bool rebalance_leaders = false;
    int64_t min_replicas = 2;
    double min_unbalance = 0.01;
    bool complete_partition = true;
    bool brokers_nil = true;
    std::vector<int64_t> brokers;
};

inline RebalanceConfig DefaultRebalanceConfig() { return RebalanceConfig(); }   // balancer.go:24-32

}  // namespace kbh

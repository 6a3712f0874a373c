// Stand-in for pitt_msgs/ClustersOutput ({cluster_objs[]}; compile checks and harness).
#pragma once
#include <memory>
#include <vector>
#include "pitt_msgs/ClusterSegmentation.h"
namespace pitt_msgs {
struct ClustersOutput {
    std::vector<InliersCluster> cluster_objs;
};
typedef std::shared_ptr<const ClustersOutput> ClustersOutputConstPtr;
}  // namespace pitt_msgs

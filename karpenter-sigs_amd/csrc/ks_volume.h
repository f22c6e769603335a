// ks_volume.h — the snapshot's PersistentVolumeClaim / PersistentVolume / StorageClass objects and the
// reference's reads of them while it builds a scheduler:
//
//   VolumeTopology.Inject     pkg/controllers/provisioning/scheduling/volumetopology.go:41-140, run by
//                             Provisioner.injectTopology before NewTopology (provisioner.go:283-284,432-442)
//   GetVolumes/resolveDriver  pkg/scheduling/volumeusage.go:82-182 (PV CSI driver, in-tree EBS, the storage
//                             class provisioner through the CSI migration name table)
//   GetPersistentVolumeClaim  pkg/utils/volume/volume.go:29-46 (claimName, or <pod>-<volume> for ephemeral)
#pragma once
#include <map>
#include <string>
#include <vector>

#include "ks_host.h"
#include "ks_json.h"

namespace ks {

struct VolumeObjects {
  struct PVC {
    std::string volumeName;  // spec.volumeName ("" = unbound)
    std::string sc;          // lo.FromPtr(spec.storageClassName) (nil and "" both read as "")
  };
  struct PV {
    std::string csiDriver;             // spec.csi.driver
    bool awsEBS = false;               // spec.awsElasticBlockStore != nil
    bool required = false;             // spec.nodeAffinity.required != nil
    std::vector<std::vector<NSR>> terms;  // its nodeSelectorTerms' matchExpressions
  };
  struct SC {
    std::string provisioner;
    bool allowed = false;    // len(allowedTopologies) > 0
    std::vector<NSR> first;  // allowedTopologies[0].matchLabelExpressions as In requirements
  };
  bool present = false;  // the snapshot carries the objects (any of the three keys)
  std::map<std::string, PVC> pvcs;  // "namespace/name"
  std::map<std::string, PV> pvs;    // by name (cluster-scoped)
  std::map<std::string, SC> scs;    // by name (cluster-scoped)

  void parse(const ksjson::Value& root);
  // VolumeTopology.Inject for one pod: false on the reference's error paths (PVC, PV or storage class not
  // found), leaving the pod unchanged -- Provisioner.injectTopology then leaves it out of NewTopology's pod
  // list (it is still scheduled); `why` gets the reference's error text.
  bool inject(PodH& p, std::string* why) const;
  // resolveDriver for one claim key (GetVolumes, volumeusage.go:87-111): returns false on the error path
  // (a bound PV that does not exist); `driver` "" = the claim is skipped (not found, no CSI driver, no class).
  bool driver(const std::string& key, std::string& out) const;
};

// csi-translation-lib v0.28.4 GetCSINameFromInTreeName: the in-tree provisioner names with a CSI migration
// driver; false for any other name (volumeusage.go:163-167 then keeps the provisioner as given).
bool csi_name_from_in_tree(const std::string& provisioner, std::string& out);

}  // namespace ks

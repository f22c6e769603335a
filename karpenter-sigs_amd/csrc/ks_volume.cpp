// ks_volume.cpp — PersistentVolumeClaim / PersistentVolume / StorageClass reads of the scheduler build
// (ks_volume.h): VolumeTopology.Inject and GetVolumes' driver resolution, from the snapshot's objects.
#include "ks_volume.h"

namespace ks {

using ksjson::Value;

namespace {

std::string vstr(const Value* v, const char* k) {
  if (!v) return "";
  const Value* x = v->get(k);
  return x && x->is_str() ? x->s : "";
}
const Value* vobj(const Value* v, const char* k) {
  if (!v) return nullptr;
  const Value* x = v->get(k);
  return x && !x->is_null() ? x : nullptr;
}
std::vector<NSR> vnsr(const Value* v) {  // []NodeSelectorRequirement
  std::vector<NSR> out;
  if (!v) return out;
  for (auto& e : v->arr()) {
    NSR n{vstr(&e, "key"), vstr(&e, "operator"), {}};
    if (auto* vs = e.get("values")) for (auto& x : vs->arr()) n.values.push_back(x.str());
    out.push_back(n);
  }
  return out;
}

}  // namespace

bool csi_name_from_in_tree(const std::string& provisioner, std::string& out) {
  // k8s.io/csi-translation-lib v0.28.4 (go.mod:30): translate.go's inTreePlugins, each plugin's
  // GetInTreePluginName -> its CSI driver name (plugins/*.go)
  static const std::pair<const char*, const char*> kTable[] = {
      {"kubernetes.io/gce-pd", "pd.csi.storage.gke.io"},
      {"kubernetes.io/aws-ebs", "ebs.csi.aws.com"},
      {"kubernetes.io/cinder", "cinder.csi.openstack.org"},
      {"kubernetes.io/azure-disk", "disk.csi.azure.com"},
      {"kubernetes.io/azure-file", "file.csi.azure.com"},
      {"kubernetes.io/vsphere-volume", "csi.vsphere.vmware.com"},
      {"kubernetes.io/portworx-volume", "pxd.portworx.com"},
      {"kubernetes.io/rbd", "rbd.csi.ceph.com"},
  };
  for (auto& e : kTable)
    if (provisioner == e.first) {
      out = e.second;
      return true;
    }
  return false;
}

void VolumeObjects::parse(const Value& root) {
  const Value* pvcV = root.get("persistentVolumeClaims");
  const Value* pvV = root.get("persistentVolumes");
  const Value* scV = root.get("storageClasses");
  present = pvcV || pvV || scV;
  if (pvcV)
    for (auto& v : pvcV->arr()) {
      const Value* md = v.get("metadata");
      const Value* sp = v.get("spec");
      pvcs[vstr(md, "namespace") + "/" + vstr(md, "name")] = PVC{vstr(sp, "volumeName"), vstr(sp, "storageClassName")};
    }
  if (pvV)
    for (auto& v : pvV->arr()) {
      const Value* sp = v.get("spec");
      PV pv;
      if (const Value* csi = vobj(sp, "csi")) pv.csiDriver = vstr(csi, "driver");
      pv.awsEBS = vobj(sp, "awsElasticBlockStore") != nullptr;
      if (const Value* req = vobj(vobj(sp, "nodeAffinity"), "required")) {
        pv.required = true;
        if (const Value* ts = req->get("nodeSelectorTerms"))
          for (auto& t : ts->arr()) pv.terms.push_back(vnsr(t.get("matchExpressions")));
      }
      pvs[vstr(v.get("metadata"), "name")] = pv;
    }
  if (scV)
    for (auto& v : scV->arr()) {
      SC sc;
      sc.provisioner = vstr(&v, "provisioner");
      if (const Value* at = v.get("allowedTopologies"); at && !at->arr().empty()) {
        sc.allowed = true;
        if (const Value* es = at->arr()[0].get("matchLabelExpressions"))
          for (auto& e : es->arr()) {  // TopologySelectorLabelRequirement -> NodeSelectorRequirement{In}
            NSR n{vstr(&e, "key"), "In", {}};
            if (auto* vs = e.get("values")) for (auto& x : vs->arr()) n.values.push_back(x.str());
            sc.first.push_back(n);
          }
      }
      scs[vstr(v.get("metadata"), "name")] = sc;
    }
}

bool VolumeObjects::inject(PodH& p, std::string* why) const {
  std::vector<NSR> reqs;
  for (const std::string& name : p.pvcNames) {  // getRequirements per volume, in spec order
    auto c = pvcs.find(p.ns + "/" + name);
    if (c == pvcs.end()) {
      if (why) *why = "discovering persistent volume claim, getting persistent volume claim \"" + name + "\"";
      return false;
    }
    if (!c->second.volumeName.empty()) {  // getPersistentVolumeRequirements: the first term only
      auto v = pvs.find(c->second.volumeName);
      if (v == pvs.end()) {
        if (why) *why = "getting existing requirements, getting persistent volume \"" + c->second.volumeName + "\"";
        return false;
      }
      if (v->second.required && !v->second.terms.empty())
        reqs.insert(reqs.end(), v->second.terms[0].begin(), v->second.terms[0].end());
      continue;
    }
    if (!c->second.sc.empty()) {  // getStorageClassRequirements: allowedTopologies[0] as In requirements
      auto s = scs.find(c->second.sc);
      if (s == scs.end()) {
        if (why) *why = "getting storage class \"" + c->second.sc + "\"";
        return false;
      }
      reqs.insert(reqs.end(), s->second.first.begin(), s->second.first.end());
    }
  }
  if (reqs.empty()) return true;
  // AND the requirements into every required node-selector term (creating one if there is none), so a
  // relaxation that drops a term cannot drop them (volumetopology.go:53-71)
  p.hasAffinity = p.hasNodeAffinity = p.hasRequired = true;
  if (p.requiredTerms.empty()) p.requiredTerms.emplace_back();
  for (auto& t : p.requiredTerms) t.insert(t.end(), reqs.begin(), reqs.end());
  return true;
}

bool VolumeObjects::driver(const std::string& key, std::string& out) const {
  out.clear();
  auto c = pvcs.find(key);
  if (c == pvcs.end()) return true;  // NotFound: the volume is ignored (volumeusage.go:88-94)
  if (!c->second.volumeName.empty()) {  // driverFromVolume
    auto v = pvs.find(c->second.volumeName);
    if (v == pvs.end()) return false;  // the PV Get error is returned (volumeusage.go:123-126)
    if (!v->second.csiDriver.empty() || v->second.awsEBS) {
      out = !v->second.csiDriver.empty() ? v->second.csiDriver : "ebs.csi.aws.com";  // plugins.AWSEBSDriverName
      return true;
    }
  }
  if (c->second.sc.empty()) return true;  // no storage class: skipped
  auto s = scs.find(c->second.sc);
  if (s == scs.end()) return true;  // a missing class: skipped (volumeusage.go:143-151)
  if (!csi_name_from_in_tree(s->second.provisioner, out)) out = s->second.provisioner;
  return true;
}

}  // namespace ks

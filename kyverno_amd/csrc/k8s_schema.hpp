// The JSON shape of the Kubernetes types the PSS handler decodes into (validate_pss.go:137-188
// getSpec: corev1.Pod; appsv1.Deployment for every controller kind; batchv1.CronJob), restated
// from k8s.io/api v0.29.1 and k8s.io/apimachinery v0.29.1 (go.mod:76,78; third-party, absent
// from the reference tree). encoding/json fails the whole decode on the first type mismatch
// anywhere in these structs (a RuleError); members not listed are ignored, as json ignores
// unknown fields. Inline members (VolumeSource, EphemeralContainerCommon, LocalObjectReference
// in key selectors) are flattened into their parent.
//
// Types: s string, b bool, i32 / i64 integers (an integer literal in range), q
// resource.Quantity (a number, or a string ParseQuantity accepts), ios intstr.IntOrString (a
// string, or an int32 literal), t metav1.Time (an RFC 3339 string), raw (any JSON: FieldsV1),
// [T] slice, {T} map[string]T, Name a struct (value or pointer: null leaves it unset).
#pragma once
#include <cctype>
#include <cstdint>
#include <functional>
#include <stdexcept>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace k8s {

inline const char* schema_text() {
  return R"K8S(
Pod{kind:s,apiVersion:s,metadata:ObjectMeta,spec:PodSpec,status:PodStatus}
Deployment{kind:s,apiVersion:s,metadata:ObjectMeta,spec:DeploymentSpec,status:DeploymentStatus}
CronJob{kind:s,apiVersion:s,metadata:ObjectMeta,spec:CronJobSpec,status:CronJobStatus}
ObjectMeta{name:s,generateName:s,namespace:s,selfLink:s,uid:s,resourceVersion:s,generation:i64,creationTimestamp:t,deletionTimestamp:t,deletionGracePeriodSeconds:i64,labels:{s},annotations:{s},ownerReferences:[OwnerReference],finalizers:[s],managedFields:[ManagedFieldsEntry]}
OwnerReference{apiVersion:s,kind:s,name:s,uid:s,controller:b,blockOwnerDeletion:b}
ManagedFieldsEntry{manager:s,operation:s,apiVersion:s,time:t,fieldsType:s,fieldsV1:raw,subresource:s}
LabelSelector{matchLabels:{s},matchExpressions:[LabelSelectorRequirement]}
LabelSelectorRequirement{key:s,operator:s,values:[s]}
PodTemplateSpec{metadata:ObjectMeta,spec:PodSpec}
PodSpec{volumes:[Volume],initContainers:[Container],containers:[Container],ephemeralContainers:[EphemeralContainer],restartPolicy:s,terminationGracePeriodSeconds:i64,activeDeadlineSeconds:i64,dnsPolicy:s,nodeSelector:{s},serviceAccountName:s,serviceAccount:s,automountServiceAccountToken:b,nodeName:s,hostNetwork:b,hostPID:b,hostIPC:b,shareProcessNamespace:b,securityContext:PodSecurityContext,imagePullSecrets:[LocalObjectReference],hostname:s,subdomain:s,affinity:Affinity,schedulerName:s,tolerations:[Toleration],hostAliases:[HostAlias],priorityClassName:s,priority:i32,dnsConfig:PodDNSConfig,readinessGates:[PodReadinessGate],runtimeClassName:s,enableServiceLinks:b,preemptionPolicy:s,overhead:{q},topologySpreadConstraints:[TopologySpreadConstraint],setHostnameAsFQDN:b,os:PodOS,hostUsers:b,schedulingGates:[PodSchedulingGate],resourceClaims:[PodResourceClaim]}
LocalObjectReference{name:s}
Toleration{key:s,operator:s,value:s,effect:s,tolerationSeconds:i64}
HostAlias{ip:s,hostnames:[s]}
PodDNSConfig{nameservers:[s],searches:[s],options:[PodDNSConfigOption]}
PodDNSConfigOption{name:s,value:s}
PodReadinessGate{conditionType:s}
TopologySpreadConstraint{maxSkew:i32,topologyKey:s,whenUnsatisfiable:s,labelSelector:LabelSelector,minDomains:i32,nodeAffinityPolicy:s,nodeTaintsPolicy:s,matchLabelKeys:[s]}
PodOS{name:s}
PodSchedulingGate{name:s}
PodResourceClaim{name:s,source:ClaimSource}
ClaimSource{resourceClaimName:s,resourceClaimTemplateName:s}
Affinity{nodeAffinity:NodeAffinity,podAffinity:PodAffinity,podAntiAffinity:PodAffinity}
NodeAffinity{requiredDuringSchedulingIgnoredDuringExecution:NodeSelector,preferredDuringSchedulingIgnoredDuringExecution:[PreferredSchedulingTerm]}
NodeSelector{nodeSelectorTerms:[NodeSelectorTerm]}
NodeSelectorTerm{matchExpressions:[NodeSelectorRequirement],matchFields:[NodeSelectorRequirement]}
NodeSelectorRequirement{key:s,operator:s,values:[s]}
PreferredSchedulingTerm{weight:i32,preference:NodeSelectorTerm}
PodAffinity{requiredDuringSchedulingIgnoredDuringExecution:[PodAffinityTerm],preferredDuringSchedulingIgnoredDuringExecution:[WeightedPodAffinityTerm]}
PodAffinityTerm{labelSelector:LabelSelector,namespaces:[s],topologyKey:s,namespaceSelector:LabelSelector,matchLabelKeys:[s],mismatchLabelKeys:[s]}
WeightedPodAffinityTerm{weight:i32,podAffinityTerm:PodAffinityTerm}
PodSecurityContext{seLinuxOptions:SELinuxOptions,windowsOptions:WindowsSecurityContextOptions,runAsUser:i64,runAsGroup:i64,runAsNonRoot:b,supplementalGroups:[i64],fsGroup:i64,sysctls:[Sysctl],fsGroupChangePolicy:s,seccompProfile:SeccompProfile}
SecurityContext{capabilities:Capabilities,privileged:b,seLinuxOptions:SELinuxOptions,windowsOptions:WindowsSecurityContextOptions,runAsUser:i64,runAsGroup:i64,runAsNonRoot:b,readOnlyRootFilesystem:b,allowPrivilegeEscalation:b,procMount:s,seccompProfile:SeccompProfile}
Capabilities{add:[s],drop:[s]}
SELinuxOptions{user:s,role:s,type:s,level:s}
WindowsSecurityContextOptions{gmsaCredentialSpecName:s,gmsaCredentialSpec:s,runAsUserName:s,hostProcess:b}
SeccompProfile{type:s,localhostProfile:s}
Sysctl{name:s,value:s}
Container{name:s,image:s,command:[s],args:[s],workingDir:s,ports:[ContainerPort],envFrom:[EnvFromSource],env:[EnvVar],resources:ResourceRequirements,resizePolicy:[ContainerResizePolicy],restartPolicy:s,volumeMounts:[VolumeMount],volumeDevices:[VolumeDevice],livenessProbe:Probe,readinessProbe:Probe,startupProbe:Probe,lifecycle:Lifecycle,terminationMessagePath:s,terminationMessagePolicy:s,imagePullPolicy:s,securityContext:SecurityContext,stdin:b,stdinOnce:b,tty:b}
EphemeralContainer{name:s,image:s,command:[s],args:[s],workingDir:s,ports:[ContainerPort],envFrom:[EnvFromSource],env:[EnvVar],resources:ResourceRequirements,resizePolicy:[ContainerResizePolicy],restartPolicy:s,volumeMounts:[VolumeMount],volumeDevices:[VolumeDevice],livenessProbe:Probe,readinessProbe:Probe,startupProbe:Probe,lifecycle:Lifecycle,terminationMessagePath:s,terminationMessagePolicy:s,imagePullPolicy:s,securityContext:SecurityContext,stdin:b,stdinOnce:b,tty:b,targetContainerName:s}
ContainerPort{name:s,hostPort:i32,containerPort:i32,protocol:s,hostIP:s}
EnvFromSource{prefix:s,configMapRef:ConfigMapEnvSource,secretRef:SecretEnvSource}
ConfigMapEnvSource{name:s,optional:b}
SecretEnvSource{name:s,optional:b}
EnvVar{name:s,value:s,valueFrom:EnvVarSource}
EnvVarSource{fieldRef:ObjectFieldSelector,resourceFieldRef:ResourceFieldSelector,configMapKeyRef:ConfigMapKeySelector,secretKeyRef:SecretKeySelector}
ObjectFieldSelector{apiVersion:s,fieldPath:s}
ResourceFieldSelector{containerName:s,resource:s,divisor:q}
ConfigMapKeySelector{name:s,key:s,optional:b}
SecretKeySelector{name:s,key:s,optional:b}
ResourceRequirements{limits:{q},requests:{q},claims:[ResourceClaim]}
ResourceClaim{name:s}
ContainerResizePolicy{resourceName:s,restartPolicy:s}
VolumeMount{name:s,readOnly:b,mountPath:s,subPath:s,mountPropagation:s,subPathExpr:s}
VolumeDevice{name:s,devicePath:s}
Probe{exec:ExecAction,httpGet:HTTPGetAction,tcpSocket:TCPSocketAction,grpc:GRPCAction,initialDelaySeconds:i32,timeoutSeconds:i32,periodSeconds:i32,successThreshold:i32,failureThreshold:i32,terminationGracePeriodSeconds:i64}
ExecAction{command:[s]}
HTTPGetAction{path:s,port:ios,host:s,scheme:s,httpHeaders:[HTTPHeader]}
HTTPHeader{name:s,value:s}
TCPSocketAction{port:ios,host:s}
GRPCAction{port:i32,service:s}
Lifecycle{postStart:LifecycleHandler,preStop:LifecycleHandler}
LifecycleHandler{exec:ExecAction,httpGet:HTTPGetAction,tcpSocket:TCPSocketAction,sleep:SleepAction}
SleepAction{seconds:i64}
Volume{name:s,hostPath:HostPathVolumeSource,emptyDir:EmptyDirVolumeSource,gcePersistentDisk:GCEPersistentDiskVolumeSource,awsElasticBlockStore:AWSElasticBlockStoreVolumeSource,gitRepo:GitRepoVolumeSource,secret:SecretVolumeSource,nfs:NFSVolumeSource,iscsi:ISCSIVolumeSource,glusterfs:GlusterfsVolumeSource,persistentVolumeClaim:PersistentVolumeClaimVolumeSource,rbd:RBDVolumeSource,flexVolume:FlexVolumeSource,cinder:CinderVolumeSource,cephfs:CephFSVolumeSource,flocker:FlockerVolumeSource,downwardAPI:DownwardAPIVolumeSource,fc:FCVolumeSource,azureFile:AzureFileVolumeSource,configMap:ConfigMapVolumeSource,vsphereVolume:VsphereVirtualDiskVolumeSource,quobyte:QuobyteVolumeSource,azureDisk:AzureDiskVolumeSource,photonPersistentDisk:PhotonPersistentDiskVolumeSource,projected:ProjectedVolumeSource,portworxVolume:PortworxVolumeSource,scaleIO:ScaleIOVolumeSource,storageos:StorageOSVolumeSource,csi:CSIVolumeSource,ephemeral:EphemeralVolumeSource}
HostPathVolumeSource{path:s,type:s}
EmptyDirVolumeSource{medium:s,sizeLimit:q}
GCEPersistentDiskVolumeSource{pdName:s,fsType:s,partition:i32,readOnly:b}
AWSElasticBlockStoreVolumeSource{volumeID:s,fsType:s,partition:i32,readOnly:b}
GitRepoVolumeSource{repository:s,revision:s,directory:s}
SecretVolumeSource{secretName:s,items:[KeyToPath],defaultMode:i32,optional:b}
KeyToPath{key:s,path:s,mode:i32}
NFSVolumeSource{server:s,path:s,readOnly:b}
ISCSIVolumeSource{targetPortal:s,iqn:s,lun:i32,iscsiInterface:s,fsType:s,readOnly:b,portals:[s],chapAuthDiscovery:b,chapAuthSession:b,secretRef:LocalObjectReference,initiatorName:s}
GlusterfsVolumeSource{endpoints:s,path:s,readOnly:b}
PersistentVolumeClaimVolumeSource{claimName:s,readOnly:b}
RBDVolumeSource{monitors:[s],image:s,fsType:s,pool:s,user:s,keyring:s,secretRef:LocalObjectReference,readOnly:b}
FlexVolumeSource{driver:s,fsType:s,secretRef:LocalObjectReference,readOnly:b,options:{s}}
CinderVolumeSource{volumeID:s,fsType:s,readOnly:b,secretRef:LocalObjectReference}
CephFSVolumeSource{monitors:[s],path:s,user:s,secretFile:s,secretRef:LocalObjectReference,readOnly:b}
FlockerVolumeSource{datasetName:s,datasetUUID:s}
DownwardAPIVolumeSource{items:[DownwardAPIVolumeFile],defaultMode:i32}
DownwardAPIVolumeFile{path:s,fieldRef:ObjectFieldSelector,resourceFieldRef:ResourceFieldSelector,mode:i32}
FCVolumeSource{targetWWNs:[s],lun:i32,fsType:s,readOnly:b,wwids:[s]}
AzureFileVolumeSource{secretName:s,shareName:s,readOnly:b}
ConfigMapVolumeSource{name:s,items:[KeyToPath],defaultMode:i32,optional:b}
VsphereVirtualDiskVolumeSource{volumePath:s,fsType:s,storagePolicyName:s,storagePolicyID:s}
QuobyteVolumeSource{registry:s,volume:s,readOnly:b,user:s,group:s,tenant:s}
AzureDiskVolumeSource{diskName:s,diskURI:s,cachingMode:s,fsType:s,readOnly:b,kind:s}
PhotonPersistentDiskVolumeSource{pdID:s,fsType:s}
ProjectedVolumeSource{sources:[VolumeProjection],defaultMode:i32}
VolumeProjection{secret:SecretProjection,downwardAPI:DownwardAPIProjection,configMap:ConfigMapProjection,serviceAccountToken:ServiceAccountTokenProjection,clusterTrustBundle:ClusterTrustBundleProjection}
SecretProjection{name:s,items:[KeyToPath],optional:b}
DownwardAPIProjection{items:[DownwardAPIVolumeFile]}
ConfigMapProjection{name:s,items:[KeyToPath],optional:b}
ServiceAccountTokenProjection{audience:s,expirationSeconds:i64,path:s}
ClusterTrustBundleProjection{name:s,signerName:s,labelSelector:LabelSelector,optional:b,path:s}
PortworxVolumeSource{volumeID:s,fsType:s,readOnly:b}
ScaleIOVolumeSource{gateway:s,system:s,secretRef:LocalObjectReference,sslEnabled:b,protectionDomain:s,storagePool:s,storageMode:s,volumeName:s,fsType:s,readOnly:b}
StorageOSVolumeSource{volumeName:s,volumeNamespace:s,fsType:s,readOnly:b,secretRef:LocalObjectReference}
CSIVolumeSource{driver:s,readOnly:b,fsType:s,volumeAttributes:{s},nodePublishSecretRef:LocalObjectReference}
EphemeralVolumeSource{volumeClaimTemplate:PersistentVolumeClaimTemplate}
PersistentVolumeClaimTemplate{metadata:ObjectMeta,spec:PersistentVolumeClaimSpec}
PersistentVolumeClaimSpec{accessModes:[s],selector:LabelSelector,resources:VolumeResourceRequirements,volumeName:s,storageClassName:s,volumeMode:s,dataSource:TypedLocalObjectReference,dataSourceRef:TypedObjectReference,volumeAttributesClassName:s}
VolumeResourceRequirements{limits:{q},requests:{q}}
TypedLocalObjectReference{apiGroup:s,kind:s,name:s}
TypedObjectReference{apiGroup:s,kind:s,name:s,namespace:s}
PodStatus{phase:s,conditions:[PodCondition],message:s,reason:s,nominatedNodeName:s,hostIP:s,hostIPs:[HostIP],podIP:s,podIPs:[PodIP],startTime:t,initContainerStatuses:[ContainerStatus],containerStatuses:[ContainerStatus],qosClass:s,ephemeralContainerStatuses:[ContainerStatus],resize:s,resourceClaimStatuses:[PodResourceClaimStatus]}
PodCondition{type:s,status:s,lastProbeTime:t,lastTransitionTime:t,reason:s,message:s}
HostIP{ip:s}
PodIP{ip:s}
ContainerStatus{name:s,state:ContainerState,lastState:ContainerState,ready:b,restartCount:i32,image:s,imageID:s,containerID:s,started:b,allocatedResources:{q},resources:ResourceRequirements}
ContainerState{waiting:ContainerStateWaiting,running:ContainerStateRunning,terminated:ContainerStateTerminated}
ContainerStateWaiting{reason:s,message:s}
ContainerStateRunning{startedAt:t}
ContainerStateTerminated{exitCode:i32,signal:i32,reason:s,message:s,startedAt:t,finishedAt:t,containerID:s}
PodResourceClaimStatus{name:s,resourceClaimName:s}
DeploymentSpec{replicas:i32,selector:LabelSelector,template:PodTemplateSpec,strategy:DeploymentStrategy,minReadySeconds:i32,revisionHistoryLimit:i32,paused:b,progressDeadlineSeconds:i32}
DeploymentStrategy{type:s,rollingUpdate:RollingUpdateDeployment}
RollingUpdateDeployment{maxUnavailable:ios,maxSurge:ios}
DeploymentStatus{observedGeneration:i64,replicas:i32,updatedReplicas:i32,readyReplicas:i32,availableReplicas:i32,unavailableReplicas:i32,conditions:[DeploymentCondition],collisionCount:i32}
DeploymentCondition{type:s,status:s,lastUpdateTime:t,lastTransitionTime:t,reason:s,message:s}
CronJobSpec{schedule:s,timeZone:s,startingDeadlineSeconds:i64,concurrencyPolicy:s,suspend:b,jobTemplate:JobTemplateSpec,successfulJobsHistoryLimit:i32,failedJobsHistoryLimit:i32}
JobTemplateSpec{metadata:ObjectMeta,spec:JobSpec}
JobSpec{parallelism:i32,completions:i32,activeDeadlineSeconds:i64,podFailurePolicy:PodFailurePolicy,backoffLimit:i32,backoffLimitPerIndex:i32,maxFailedIndexes:i32,selector:LabelSelector,manualSelector:b,template:PodTemplateSpec,ttlSecondsAfterFinished:i32,completionMode:s,suspend:b,podReplacementPolicy:s}
PodFailurePolicy{rules:[PodFailurePolicyRule]}
PodFailurePolicyRule{action:s,onExitCodes:PodFailurePolicyOnExitCodesRequirement,onPodConditions:[PodFailurePolicyOnPodConditionsPattern]}
PodFailurePolicyOnExitCodesRequirement{containerName:s,operator:s,values:[i32]}
PodFailurePolicyOnPodConditionsPattern{type:s,status:s}
CronJobStatus{active:[ObjectReference],lastScheduleTime:t,lastSuccessfulTime:t}
ObjectReference{kind:s,namespace:s,name:s,uid:s,apiVersion:s,resourceVersion:s,fieldPath:s}
)K8S";
}

enum Kind : uint8_t { K_STR, K_BOOL, K_I32, K_I64, K_QTY, K_IOS, K_TIME, K_RAW, K_STRUCT, K_LIST, K_MAP };
struct Type {
  Kind kind;
  uint16_t sub;  // K_STRUCT: struct index; K_LIST / K_MAP: element type index
};
struct Field {
  std::string lower;  // json name, lower-cased (encoding/json matches case-insensitively)
  std::string exact;
  uint16_t type;
};
struct Struct {
  std::string name;
  std::vector<Field> fields;
};
struct Schema {
  std::vector<Type> types;
  std::vector<Struct> structs;
  std::unordered_map<std::string, uint16_t> by_name;
  // the field of struct s for json key k: an exact match first, else case-insensitive (-1: none)
  int field(uint16_t s, std::string_view k) const {
    const auto& F = structs[s].fields;
    for (size_t i = 0; i < F.size(); ++i)
      if (F[i].exact == k) return (int)i;
    for (size_t i = 0; i < F.size(); ++i) {
      const std::string& l = F[i].lower;
      if (l.size() != k.size()) continue;
      bool eq = true;
      for (size_t j = 0; j < k.size() && eq; ++j) eq = l[j] == (char)std::tolower((unsigned char)k[j]);
      if (eq) return (int)i;
    }
    return -1;
  }
  uint16_t struct_id(const std::string& n) const { return by_name.at(n); }
};

inline const Schema& schema() {
  static const Schema S = [] {
    Schema s;
    const std::string txt = schema_text();
    // pass 1: struct names
    for (size_t i = 0; i < txt.size();) {
      size_t e = txt.find('\n', i);
      if (e == std::string::npos) e = txt.size();
      const std::string line = txt.substr(i, e - i);
      i = e + 1;
      const size_t b = line.find('{');
      if (b == std::string::npos) continue;
      s.by_name[line.substr(0, b)] = (uint16_t)s.structs.size();
      s.structs.push_back(Struct{line.substr(0, b), {}});
    }
    std::unordered_map<std::string, uint16_t> memo;
    std::function<uint16_t(const std::string&)> ty = [&](const std::string& t) -> uint16_t {
      auto it = memo.find(t);
      if (it != memo.end()) return it->second;
      Type x{K_STR, 0};
      if (t == "s") x.kind = K_STR;
      else if (t == "b") x.kind = K_BOOL;
      else if (t == "i32") x.kind = K_I32;
      else if (t == "i64") x.kind = K_I64;
      else if (t == "q") x.kind = K_QTY;
      else if (t == "ios") x.kind = K_IOS;
      else if (t == "t") x.kind = K_TIME;
      else if (t == "raw") x.kind = K_RAW;
      else if (t.front() == '[') x.kind = K_LIST, x.sub = ty(t.substr(1, t.size() - 2));
      else if (t.front() == '{') x.kind = K_MAP, x.sub = ty(t.substr(1, t.size() - 2));
      else {
        auto st = s.by_name.find(t);
        if (st == s.by_name.end()) throw std::logic_error("k8s schema: unknown type " + t);
        x.kind = K_STRUCT, x.sub = st->second;
      }
      s.types.push_back(x);
      return memo[t] = (uint16_t)(s.types.size() - 1);
    };
    // pass 2: fields
    for (auto& st : s.structs) {  // one struct per line: Name{...}
      const size_t at = txt.find("\n" + st.name + "{");
      const size_t b = at + st.name.size() + 2, e = txt.find('\n', b) - 1;
      std::string body = txt.substr(b, e - b);
      size_t p = 0;
      while (p < body.size()) {
        size_t c = body.find(':', p);
        // a field's type may itself contain ',' only inside [] / {}: scan to the next top-level ','
        size_t q = c + 1;
        int depth = 0;
        while (q < body.size() && (depth > 0 || body[q] != ',')) {
          if (body[q] == '[' || body[q] == '{') ++depth;
          if (body[q] == ']' || body[q] == '}') --depth;
          ++q;
        }
        Field f;
        f.exact = body.substr(p, c - p);
        f.lower = f.exact;
        for (auto& ch : f.lower) ch = (char)std::tolower((unsigned char)ch);
        f.type = ty(body.substr(c + 1, q - c - 1));
        st.fields.push_back(f);
        p = q + 1;
      }
    }
    return s;
  }();
  return S;
}

}  // namespace k8s

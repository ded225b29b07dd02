"""The API's type table in a compact form, expanded by `openapi.py` into OpenAPI v2 definitions
(the reference publishes the same surface as api/openapi-spec/swagger.json, generated from the
Go structs in staging/src/k8s.io/api/*/types.go; the fork's device-granular fields are in
core/v1/types.go:2204 Container.extendedResourceRequests, :2885 PodSpec.extendedResources,
:3850 NodeStatus.extendedResources, :4018-4057 the ExtendedResource* types, :4495
ObjectReference.extendedResourceBinding).

Grammar (one definition per block):

    @<definition prefix>                 sets the prefix of the definitions that follow
    Name [+kind] [description]           a definition; +kind adds apiVersion, kind, metadata
      field type[!] [description]        a property; ! marks it required

Types: string integer long boolean number byte time quantity ios object, another definition's
short name (or a full definition id), []T for arrays and {}T for string-keyed maps.
Descriptions are this project's own wording.
"""

TYPES = r"""
@io.k8s.apimachinery.pkg.apis.meta.v1
ObjectMeta  Metadata every persisted object carries.
  name string  Unique name within the namespace; used in URLs; cannot be changed.
  generateName string  Prefix from which the server generates a unique name when name is empty.
  namespace string  Namespace the object lives in; empty for cluster-scoped objects.
  selfLink string  Read-only URL of the object.
  uid string  Read-only identifier unique over the cluster's lifetime.
  resourceVersion string  Opaque version used for optimistic concurrency and watches.
  generation long  Sequence number of the desired state; set by the system.
  creationTimestamp time  Read-only server time of creation.
  deletionTimestamp time  Time after which the object will be removed; set by a graceful delete.
  deletionGracePeriodSeconds long  Seconds the object is given to terminate before it is removed.
  labels {}string  Key/value pairs used to select and organise objects.
  annotations {}string  Unstructured key/value data tools attach to the object.
  ownerReferences []OwnerReference  Objects this one depends on; the garbage collector deletes it when all owners are gone.
  initializers Initializers  Pending initializers; the object is hidden from normal reads until the list is empty.
  finalizers []string  Entries that must be cleared before the object is removed from storage.
  clusterName string  Name of the cluster the object belongs to.
ListMeta  Metadata of a list response.
  selfLink string  Read-only URL of the list.
  resourceVersion string  Version of the list; start a watch from here.
  continue string  Token that fetches the next chunk of a paginated list.
OwnerReference  Identifies an owning object.
  apiVersion string!  API version of the owner.
  kind string!  Kind of the owner.
  name string!  Name of the owner.
  uid string!  UID of the owner.
  controller boolean  True when the owner is the managing controller.
  blockOwnerDeletion boolean  When true, the owner cannot be deleted in foreground until this reference is removed.
Initializers  Pending and failed initialization of an object.
  pending []Initializer!  Initializers that still have to act, in order.
  result Status  Set when initialization failed; the object is then deleted.
Initializer  One pending initializer.
  name string!  Name of the process that performs the initialization.
LabelSelector  Label query over a set of objects; the requirements are ANDed.
  matchLabels {}string  Equality requirements.
  matchExpressions []LabelSelectorRequirement  Set-based requirements.
LabelSelectorRequirement  One set-based label requirement.
  key string!  Label key.
  operator string!  In, NotIn, Exists or DoesNotExist.
  values []string  Values for In and NotIn.
Time  RFC 3339 timestamp with second precision.
Status  Result of an operation that does not return an object.
  apiVersion string  Versioned schema of this representation.
  kind string  Always Status.
  metadata ListMeta
  status string  Success or Failure.
  message string  Human-readable description.
  reason string  Machine-readable reason (NotFound, AlreadyExists, Conflict, ...).
  details StatusDetails  Extra data about the reason.
  code integer  HTTP status code.
StatusDetails  Extra data of a Status.
  name string
  group string
  kind string
  uid string
  causes []StatusCause
  retryAfterSeconds integer
StatusCause  One cause of an error.
  reason string
  message string
  field string  Path of the field that caused the error.
DeleteOptions  Options of a DELETE.
  apiVersion string
  kind string
  gracePeriodSeconds long  Seconds before the object is deleted; 0 deletes immediately.
  preconditions Preconditions  Must hold for the delete to proceed.
  orphanDependents boolean  Deprecated; use propagationPolicy.
  propagationPolicy string  Orphan, Background or Foreground garbage collection of dependents.
Preconditions  Conditions a DELETE checks.
  uid string
WatchEvent  One event of a watch stream.
  type string!  ADDED, MODIFIED, DELETED or ERROR.
  object io.k8s.apimachinery.pkg.runtime.RawExtension!  The object (or a Status for ERROR).
APIResource  One resource of a group version.
  name string!
  singularName string!
  namespaced boolean!
  group string
  version string
  kind string!
  verbs []string!
  shortNames []string
  categories []string
APIResourceList  Resources served by one group version.
  apiVersion string
  kind string
  groupVersion string!
  resources []APIResource!
APIGroup  One API group and its versions.
  apiVersion string
  kind string
  name string!
  versions []GroupVersionForDiscovery!
  preferredVersion GroupVersionForDiscovery
  serverAddressByClientCIDRs []ServerAddressByClientCIDR!
APIGroupList  All API groups.
  apiVersion string
  kind string
  groups []APIGroup!
GroupVersionForDiscovery  A group version as discovery shows it.
  groupVersion string!
  version string!
ServerAddressByClientCIDR  Server address to use for clients in a CIDR.
  clientCIDR string!
  serverAddress string!
APIVersions  Versions of the legacy core API.
  apiVersion string
  kind string
  versions []string!
  serverAddressByClientCIDRs []ServerAddressByClientCIDR!

@io.k8s.api.core.v1
Pod +kind  A group of containers that share network, IPC and volumes and are scheduled onto one node together.
  spec PodSpec  Desired behaviour of the pod.
  status PodStatus  Most recently observed state of the pod; read-only.
PodSpec  Desired behaviour of a pod.
  volumes []Volume  Volumes the pod's containers can mount.
  initContainers []Container  Containers run to completion, one after another, before the app containers start.
  containers []Container!  The pod's application containers; at least one.
  restartPolicy string  Always, OnFailure or Never; default Always.
  terminationGracePeriodSeconds long  Seconds between the termination signal and the kill; default 30.
  activeDeadlineSeconds long  Seconds the pod may be active before the kubelet fails it.
  dnsPolicy string  ClusterFirst, ClusterFirstWithHostNet, Default or None.
  nodeSelector {}string  Labels a node must carry for the pod to fit.
  serviceAccountName string  Service account the pod runs as.
  serviceAccount string  Deprecated alias of serviceAccountName.
  automountServiceAccountToken boolean  Whether the service account token is mounted.
  nodeName string  Node the pod is bound to; set by the scheduler.
  hostNetwork boolean  Use the node's network namespace.
  hostPID boolean  Use the node's PID namespace.
  hostIPC boolean  Use the node's IPC namespace.
  securityContext PodSecurityContext  Pod-level security attributes.
  imagePullSecrets []LocalObjectReference  Secrets used to pull the images.
  hostname string  Pod hostname; defaults to the pod name.
  subdomain string  DNS subdomain; the pod's FQDN is hostname.subdomain.namespace.svc.<domain>.
  affinity Affinity  Node and pod (anti-)affinity scheduling constraints.
  schedulerName string  Scheduler that schedules the pod.
  tolerations []Toleration  Taints the pod tolerates.
  hostAliases []HostAlias  Extra /etc/hosts entries.
  priorityClassName string  PriorityClass that gives the pod its priority.
  priority integer  Priority value resolved from priorityClassName by admission.
  dnsConfig PodDNSConfig  Extra resolver settings merged into the generated resolv.conf.
  extendedResources []PodExtendedResource  Device-granular requests (fork): each entry names a resource, its count and an affinity over device attributes.
PodStatus  Observed state of a pod.
  phase string  Pending, Running, Succeeded, Failed or Unknown.
  conditions []PodCondition  PodScheduled, Initialized, Ready.
  message string  Why the pod is in its condition.
  reason string  Brief CamelCase reason (Evicted, ...).
  hostIP string  IP of the node the pod runs on.
  podIP string  IP of the pod.
  startTime time  When the kubelet acknowledged the pod.
  initContainerStatuses []ContainerStatus
  containerStatuses []ContainerStatus
  qosClass string  Guaranteed, Burstable or BestEffort.
PodCondition  One condition of a pod.
  type string!
  status string!  True, False or Unknown.
  lastProbeTime time
  lastTransitionTime time
  reason string
  message string
ContainerStatus  Observed state of one container.
  name string!
  state ContainerState
  lastState ContainerState  State of the previous instance.
  ready boolean!
  restartCount integer!
  image string!
  imageID string!
  containerID string  runtime://id of the container.
ContainerState  Exactly one of the members is set.
  waiting ContainerStateWaiting
  running ContainerStateRunning
  terminated ContainerStateTerminated
ContainerStateWaiting  Not yet running.
  reason string
  message string
ContainerStateRunning  Running.
  startedAt time
ContainerStateTerminated  Exited.
  exitCode integer!
  signal integer
  reason string
  message string
  startedAt time
  finishedAt time
  containerID string
Container  One container of a pod.
  name string!  DNS label, unique within the pod.
  image string  Image reference.
  command []string  Entrypoint; $(VAR) references are expanded.
  args []string  Arguments to the entrypoint.
  workingDir string
  ports []ContainerPort  Ports the container exposes.
  envFrom []EnvFromSource  Sources whose keys become environment variables.
  env []EnvVar  Environment variables.
  resources ResourceRequirements  Compute resources (cpu, memory, ephemeral-storage, amd.com/gpu, ...).
  volumeMounts []VolumeMount
  volumeDevices []VolumeDevice  Block devices from volumes (alpha).
  livenessProbe Probe
  readinessProbe Probe
  lifecycle Lifecycle
  terminationMessagePath string
  terminationMessagePolicy string  File or FallbackToLogsOnError.
  imagePullPolicy string  Always, Never or IfNotPresent.
  securityContext SecurityContext
  stdin boolean
  stdinOnce boolean
  tty boolean
  extendedResourceRequests []string  Names of the pod's extendedResources this container uses (fork).
ContainerPort  A port of a container.
  name string
  hostPort integer  Port on the node that forwards to this one.
  containerPort integer!
  protocol string  TCP or UDP.
  hostIP string
EnvVar  One environment variable.
  name string!
  value string
  valueFrom EnvVarSource
EnvVarSource  Where an environment variable's value comes from.
  fieldRef ObjectFieldSelector
  resourceFieldRef ResourceFieldSelector
  configMapKeyRef ConfigMapKeySelector
  secretKeyRef SecretKeySelector
ObjectFieldSelector  A field of the pod.
  apiVersion string
  fieldPath string!
ResourceFieldSelector  A resource limit or request of a container.
  containerName string
  resource string!
  divisor quantity
ConfigMapKeySelector  A key of a ConfigMap.
  name string
  key string!
  optional boolean
SecretKeySelector  A key of a Secret.
  name string
  key string!
  optional boolean
EnvFromSource  A ConfigMap or Secret whose keys become variables.
  prefix string
  configMapRef ConfigMapEnvSource
  secretRef SecretEnvSource
ConfigMapEnvSource  A ConfigMap for envFrom.
  name string
  optional boolean
SecretEnvSource  A Secret for envFrom.
  name string
  optional boolean
ResourceRequirements  Requests and limits of compute resources.
  limits {}quantity
  requests {}quantity
VolumeMount  A volume mounted into a container.
  name string!
  readOnly boolean
  mountPath string!
  subPath string
  mountPropagation string  HostToContainer or Bidirectional.
VolumeDevice  A block volume exposed as a device.
  name string!
  devicePath string!
Probe  A health check.
  exec ExecAction
  httpGet HTTPGetAction
  tcpSocket TCPSocketAction
  initialDelaySeconds integer
  timeoutSeconds integer
  periodSeconds integer
  successThreshold integer
  failureThreshold integer
Handler  The action of a hook.
  exec ExecAction
  httpGet HTTPGetAction
  tcpSocket TCPSocketAction
ExecAction  Run a command in the container.
  command []string
HTTPGetAction  An HTTP GET.
  path string
  port ios!
  host string
  scheme string
  httpHeaders []HTTPHeader
HTTPHeader  One request header.
  name string!
  value string!
TCPSocketAction  A TCP connect.
  port ios!
  host string
Lifecycle  Hooks run by the kubelet.
  postStart Handler
  preStop Handler
SecurityContext  Container-level security attributes.
  capabilities Capabilities
  privileged boolean
  seLinuxOptions SELinuxOptions
  runAsUser long
  runAsNonRoot boolean
  readOnlyRootFilesystem boolean
  allowPrivilegeEscalation boolean
Capabilities  Linux capabilities to add or drop.
  add []string
  drop []string
SELinuxOptions  SELinux label.
  user string
  role string
  type string
  level string
PodSecurityContext  Pod-level security attributes.
  seLinuxOptions SELinuxOptions
  runAsUser long
  runAsNonRoot boolean
  supplementalGroups []long
  fsGroup long
Affinity  Scheduling constraints.
  nodeAffinity NodeAffinity
  podAffinity PodAffinity
  podAntiAffinity PodAntiAffinity
NodeAffinity  Constraints on the node's labels.
  requiredDuringSchedulingIgnoredDuringExecution NodeSelector
  preferredDuringSchedulingIgnoredDuringExecution []PreferredSchedulingTerm
NodeSelector  ORed node selector terms.
  nodeSelectorTerms []NodeSelectorTerm!
NodeSelectorTerm  ANDed requirements.
  matchExpressions []NodeSelectorRequirement!
NodeSelectorRequirement  One node label requirement.
  key string!
  operator string!  In, NotIn, Exists, DoesNotExist, Gt or Lt.
  values []string
PreferredSchedulingTerm  A weighted node preference.
  weight integer!
  preference NodeSelectorTerm!
PodAffinity  Co-locate with pods.
  requiredDuringSchedulingIgnoredDuringExecution []PodAffinityTerm
  preferredDuringSchedulingIgnoredDuringExecution []WeightedPodAffinityTerm
PodAntiAffinity  Keep away from pods.
  requiredDuringSchedulingIgnoredDuringExecution []PodAffinityTerm
  preferredDuringSchedulingIgnoredDuringExecution []WeightedPodAffinityTerm
PodAffinityTerm  Pods matching the selector in the topology domain.
  labelSelector LabelSelector
  namespaces []string
  topologyKey string!
WeightedPodAffinityTerm  A weighted pod affinity term.
  weight integer!
  podAffinityTerm PodAffinityTerm!
Toleration  Tolerates a taint.
  key string
  operator string  Exists or Equal.
  value string
  effect string  NoSchedule, PreferNoSchedule or NoExecute.
  tolerationSeconds long  How long a NoExecute taint is tolerated.
HostAlias  One /etc/hosts entry.
  ip string
  hostnames []string
PodDNSConfig  Resolver settings.
  nameservers []string
  searches []string
  options []PodDNSConfigOption
PodDNSConfigOption  One resolver option.
  name string
  value string
PodExtendedResource  A device-granular request of a pod (fork).
  name string  Name of the request, referenced by containers' extendedResourceRequests.
  resources ResourceRequirements  Count of devices of one resource (a single entry).
  affinity ExtendedResourceAffinity  Requirements over the devices' attributes.
  annotations {}string
  assigned []string  Device IDs the scheduler bound to this request.
ResourceSelector  A requirement on a device attribute (the fork's alias of NodeSelectorRequirement).
  key string!  Attribute name, e.g. amd.com/gpu-memory.
  operator string!  In, NotIn, Exists, DoesNotExist, Gt or Lt.
  values []string  Values for In/NotIn; a single integer for Gt/Lt.
ExtendedResourceAffinity  Device attribute requirements (fork).
  required []ResourceSelector
ExtendedResourceDomain  Devices of one resource on a node (fork).
  resources {}ExtendedResource
ExtendedResource  One device (fork).
  id string
  health string  Healthy or Unhealthy.
  attributes {}string
ExtendedResourceList  Device IDs bound to one request (fork).
  resources []string
LocalObjectReference  Names an object in the same namespace.
  name string
ObjectReference  Reference to any object.
  kind string
  namespace string
  name string
  uid string
  apiVersion string
  resourceVersion string
  fieldPath string
  extendedResourceBinding {}ExtendedResourceList  Devices bound with the pod, per extended-resource request (fork).
SecretReference  A Secret in any namespace.
  name string
  namespace string
Volume  A named volume; exactly one source is set.
  name string!
  hostPath HostPathVolumeSource
  emptyDir EmptyDirVolumeSource
  gcePersistentDisk GCEPersistentDiskVolumeSource
  awsElasticBlockStore AWSElasticBlockStoreVolumeSource
  gitRepo GitRepoVolumeSource
  secret SecretVolumeSource
  nfs NFSVolumeSource
  iscsi ISCSIVolumeSource
  glusterfs GlusterfsVolumeSource
  persistentVolumeClaim PersistentVolumeClaimVolumeSource
  rbd RBDVolumeSource
  flexVolume FlexVolumeSource
  cinder CinderVolumeSource
  cephfs CephFSVolumeSource
  flocker FlockerVolumeSource
  downwardAPI DownwardAPIVolumeSource
  fc FCVolumeSource
  azureFile AzureFileVolumeSource
  configMap ConfigMapVolumeSource
  vsphereVolume VsphereVirtualDiskVolumeSource
  quobyte QuobyteVolumeSource
  azureDisk AzureDiskVolumeSource
  photonPersistentDisk PhotonPersistentDiskVolumeSource
  projected ProjectedVolumeSource
  portworxVolume PortworxVolumeSource
  scaleIO ScaleIOVolumeSource
  storageos StorageOSVolumeSource
HostPathVolumeSource  A path on the node.
  path string!
  type string  "", DirectoryOrCreate, Directory, FileOrCreate, File, Socket, CharDevice or BlockDevice.
EmptyDirVolumeSource  Scratch space that lives as long as the pod.
  medium string  "" (node disk), Memory (tmpfs) or HugePages.
  sizeLimit quantity
GCEPersistentDiskVolumeSource  A GCE persistent disk.
  pdName string!
  fsType string
  partition integer
  readOnly boolean
AWSElasticBlockStoreVolumeSource  An AWS EBS volume.
  volumeID string!
  fsType string
  partition integer
  readOnly boolean
GitRepoVolumeSource  A git checkout.
  repository string!
  revision string
  directory string
SecretVolumeSource  A Secret's keys as files.
  secretName string
  items []KeyToPath
  defaultMode integer
  optional boolean
KeyToPath  One key projected to a path.
  key string!
  path string!
  mode integer
NFSVolumeSource  An NFS export.
  server string!
  path string!
  readOnly boolean
ISCSIVolumeSource  An iSCSI LUN.
  targetPortal string!
  iqn string!
  lun integer!
  iscsiInterface string
  fsType string
  readOnly boolean
  portals []string
  chapAuthDiscovery boolean
  chapAuthSession boolean
  secretRef LocalObjectReference
  initiatorName string
ISCSIPersistentVolumeSource  An iSCSI LUN of a PersistentVolume.
  targetPortal string!
  iqn string!
  lun integer!
  iscsiInterface string
  fsType string
  readOnly boolean
  portals []string
  chapAuthDiscovery boolean
  chapAuthSession boolean
  secretRef SecretReference
  initiatorName string
GlusterfsVolumeSource  A GlusterFS volume.
  endpoints string!
  path string!
  readOnly boolean
PersistentVolumeClaimVolumeSource  A claim in the pod's namespace.
  claimName string!
  readOnly boolean
RBDVolumeSource  A Ceph RBD image.
  monitors []string!
  image string!
  fsType string
  pool string
  user string
  keyring string
  secretRef LocalObjectReference
  readOnly boolean
RBDPersistentVolumeSource  A Ceph RBD image of a PersistentVolume.
  monitors []string!
  image string!
  fsType string
  pool string
  user string
  keyring string
  secretRef SecretReference
  readOnly boolean
FlexVolumeSource  A volume handled by a FlexVolume driver.
  driver string!
  fsType string
  secretRef LocalObjectReference
  readOnly boolean
  options {}string
CinderVolumeSource  An OpenStack Cinder volume.
  volumeID string!
  fsType string
  readOnly boolean
CephFSVolumeSource  A CephFS mount.
  monitors []string!
  path string
  user string
  secretFile string
  secretRef LocalObjectReference
  readOnly boolean
CephFSPersistentVolumeSource  A CephFS mount of a PersistentVolume.
  monitors []string!
  path string
  user string
  secretFile string
  secretRef SecretReference
  readOnly boolean
FlockerVolumeSource  A Flocker dataset.
  datasetName string
  datasetUUID string
DownwardAPIVolumeSource  Pod fields as files.
  items []DownwardAPIVolumeFile
  defaultMode integer
DownwardAPIVolumeFile  One downward API file.
  path string!
  fieldRef ObjectFieldSelector
  resourceFieldRef ResourceFieldSelector
  mode integer
FCVolumeSource  A Fibre Channel volume.
  targetWWNs []string
  lun integer
  fsType string
  readOnly boolean
  wwids []string
AzureFileVolumeSource  An Azure File share.
  secretName string!
  shareName string!
  readOnly boolean
AzureFilePersistentVolumeSource  An Azure File share of a PersistentVolume.
  secretName string!
  shareName string!
  readOnly boolean
  secretNamespace string
ConfigMapVolumeSource  A ConfigMap's keys as files.
  name string
  items []KeyToPath
  defaultMode integer
  optional boolean
VsphereVirtualDiskVolumeSource  A vSphere VMDK.
  volumePath string!
  fsType string
  storagePolicyName string
  storagePolicyID string
QuobyteVolumeSource  A Quobyte volume.
  registry string!
  volume string!
  readOnly boolean
  user string
  group string
AzureDiskVolumeSource  An Azure data disk.
  diskName string!
  diskURI string!
  cachingMode string
  fsType string
  readOnly boolean
  kind string
PhotonPersistentDiskVolumeSource  A Photon Controller disk.
  pdID string!
  fsType string
ProjectedVolumeSource  Several sources in one directory.
  sources []VolumeProjection!
  defaultMode integer
VolumeProjection  One projected source.
  secret SecretProjection
  downwardAPI DownwardAPIProjection
  configMap ConfigMapProjection
SecretProjection  Keys of a Secret.
  name string
  items []KeyToPath
  optional boolean
ConfigMapProjection  Keys of a ConfigMap.
  name string
  items []KeyToPath
  optional boolean
DownwardAPIProjection  Downward API files.
  items []DownwardAPIVolumeFile
PortworxVolumeSource  A Portworx volume.
  volumeID string!
  fsType string
  readOnly boolean
ScaleIOVolumeSource  A ScaleIO volume.
  gateway string!
  system string!
  secretRef LocalObjectReference!
  sslEnabled boolean
  protectionDomain string
  storagePool string
  storageMode string
  volumeName string
  fsType string
  readOnly boolean
ScaleIOPersistentVolumeSource  A ScaleIO volume of a PersistentVolume.
  gateway string!
  system string!
  secretRef SecretReference!
  sslEnabled boolean
  protectionDomain string
  storagePool string
  storageMode string
  volumeName string
  fsType string
  readOnly boolean
StorageOSVolumeSource  A StorageOS volume.
  volumeName string
  volumeNamespace string
  fsType string
  readOnly boolean
  secretRef LocalObjectReference
StorageOSPersistentVolumeSource  A StorageOS volume of a PersistentVolume.
  volumeName string
  volumeNamespace string
  fsType string
  readOnly boolean
  secretRef ObjectReference
LocalVolumeSource  A local disk or directory of one node.
  path string!
CSIPersistentVolumeSource  A volume of a CSI driver.
  driver string!
  volumeHandle string!
  readOnly boolean
PersistentVolume +kind  A piece of storage provisioned by an administrator or a provisioner.
  spec PersistentVolumeSpec
  status PersistentVolumeStatus
PersistentVolumeSpec  What a PersistentVolume is.
  capacity {}quantity
  gcePersistentDisk GCEPersistentDiskVolumeSource
  awsElasticBlockStore AWSElasticBlockStoreVolumeSource
  hostPath HostPathVolumeSource
  glusterfs GlusterfsVolumeSource
  nfs NFSVolumeSource
  rbd RBDPersistentVolumeSource
  iscsi ISCSIPersistentVolumeSource
  cinder CinderVolumeSource
  cephfs CephFSPersistentVolumeSource
  fc FCVolumeSource
  flocker FlockerVolumeSource
  flexVolume FlexVolumeSource
  azureFile AzureFilePersistentVolumeSource
  vsphereVolume VsphereVirtualDiskVolumeSource
  quobyte QuobyteVolumeSource
  azureDisk AzureDiskVolumeSource
  photonPersistentDisk PhotonPersistentDiskVolumeSource
  portworxVolume PortworxVolumeSource
  scaleIO ScaleIOPersistentVolumeSource
  local LocalVolumeSource
  storageos StorageOSPersistentVolumeSource
  csi CSIPersistentVolumeSource
  accessModes []string  ReadWriteOnce, ReadOnlyMany or ReadWriteMany.
  claimRef ObjectReference  The claim bound to this volume.
  persistentVolumeReclaimPolicy string  Retain, Recycle or Delete.
  storageClassName string
  mountOptions []string
  volumeMode string  Filesystem or Block.
PersistentVolumeStatus  Observed state of a PersistentVolume.
  phase string  Pending, Available, Bound, Released or Failed.
  message string
  reason string
PersistentVolumeClaim +kind  A user's request for storage.
  spec PersistentVolumeClaimSpec
  status PersistentVolumeClaimStatus
PersistentVolumeClaimSpec  What a claim asks for.
  accessModes []string
  selector LabelSelector
  resources ResourceRequirements
  volumeName string  Binds the claim to this volume.
  storageClassName string
  volumeMode string
PersistentVolumeClaimStatus  Observed state of a claim.
  phase string  Pending, Bound or Lost.
  accessModes []string
  capacity {}quantity
  conditions []PersistentVolumeClaimCondition
PersistentVolumeClaimCondition  One condition of a claim.
  type string!
  status string!
  lastProbeTime time
  lastTransitionTime time
  reason string
  message string
Node +kind  A worker machine; MI355X nodes report their GPUs as extended resources.
  spec NodeSpec
  status NodeStatus
NodeSpec  Desired state of a node.
  podCIDR string
  externalID string
  providerID string
  unschedulable boolean
  taints []Taint
  configSource NodeConfigSource  Dynamic kubelet configuration source.
NodeConfigSource  Where a kubelet's configuration comes from.
  apiVersion string
  kind string
  configMapRef ObjectReference
Taint  Repels pods that do not tolerate it.
  key string!
  value string
  effect string!
  timeAdded time
NodeStatus  Observed state of a node.
  capacity {}quantity
  allocatable {}quantity
  phase string
  conditions []NodeCondition
  addresses []NodeAddress
  daemonEndpoints NodeDaemonEndpoints
  nodeInfo NodeSystemInfo
  images []ContainerImage
  volumesInUse []string
  volumesAttached []AttachedVolume
  extendedResources {}ExtendedResourceDomain  Devices of every extended resource with their health and attributes (fork).
NodeCondition  One condition of a node.
  type string!
  status string!
  lastHeartbeatTime time
  lastTransitionTime time
  reason string
  message string
NodeAddress  One address of a node.
  type string!  Hostname, ExternalIP, InternalIP, ExternalDNS or InternalDNS.
  address string!
NodeDaemonEndpoints  Ports of the node's daemons.
  kubeletEndpoint DaemonEndpoint
DaemonEndpoint  One daemon port.
  Port integer!
NodeSystemInfo  Identity of a node's software.
  machineID string!
  systemUUID string!
  bootID string!
  kernelVersion string!
  osImage string!
  containerRuntimeVersion string!
  kubeletVersion string!
  kubeProxyVersion string!
  operatingSystem string!
  architecture string!
ContainerImage  An image present on a node.
  names []string!
  sizeBytes long
AttachedVolume  A volume attached to a node.
  name string!
  devicePath string!
Binding +kind  Binds a pod to a node; the device IDs travel in target.extendedResourceBinding.
  target ObjectReference!
Event +kind +meta!  A report of something that happened in the cluster.
  involvedObject ObjectReference!
  reason string
  message string
  source EventSource
  firstTimestamp time
  lastTimestamp time
  count integer
  type string  Normal or Warning.
  eventTime microtime  When the event was first observed (events.k8s.io series).
  series EventSeries  Data about the series this event belongs to; absent for a singleton.
  action string  What was taken or failed regarding the involved object.
  related ObjectReference  A secondary object the event is about.
  reportingComponent string  Controller that emitted the event, e.g. kubernetes.io/kubelet.
  reportingInstance string  ID of that controller instance, e.g. kubelet-xyzf.
EventSeries  A series of events: something that kept happening.
  count integer  Occurrences in the series up to the last heartbeat.
  lastObservedTime microtime  Last occurrence observed.
  state string  Ongoing or Finished.
EventSource  Who reported an event.
  component string
  host string
Namespace +kind  A scope for names.
  spec NamespaceSpec
  status NamespaceStatus
NamespaceSpec  Finalizers of a namespace.
  finalizers []string
NamespaceStatus  Phase of a namespace.
  phase string  Active or Terminating.
Service +kind  A named set of pod endpoints behind one virtual address.
  spec ServiceSpec
  status ServiceStatus
ServiceSpec  What a service exposes.
  ports []ServicePort
  selector {}string
  clusterIP string  None for a headless service.
  type string  ClusterIP, NodePort, LoadBalancer or ExternalName.
  externalIPs []string
  sessionAffinity string  None or ClientIP.
  loadBalancerIP string
  loadBalancerSourceRanges []string
  externalName string
  externalTrafficPolicy string  Cluster or Local.
  healthCheckNodePort integer
  publishNotReadyAddresses boolean
  sessionAffinityConfig SessionAffinityConfig
ServicePort  One port of a service.
  name string
  protocol string
  port integer!
  targetPort ios
  nodePort integer
SessionAffinityConfig  Session affinity settings.
  clientIP ClientIPConfig
ClientIPConfig  ClientIP affinity settings.
  timeoutSeconds integer
ServiceStatus  Observed state of a service.
  loadBalancer LoadBalancerStatus
LoadBalancerStatus  Load-balancer ingress points.
  ingress []LoadBalancerIngress
LoadBalancerIngress  One ingress point.
  ip string
  hostname string
Endpoints +kind  The addresses behind a service.
  subsets []EndpointSubset!
EndpointSubset  Addresses sharing a set of ports.
  addresses []EndpointAddress
  notReadyAddresses []EndpointAddress
  ports []EndpointPort
EndpointAddress  One endpoint.
  ip string!
  hostname string
  nodeName string
  targetRef ObjectReference
EndpointPort  One endpoint port.
  name string
  port integer!
  protocol string
ConfigMap +kind  Non-secret configuration data.
  data {}string
Secret +kind  Sensitive data.
  data {}byte  Base64-encoded values.
  stringData {}string  Write-only plain values merged into data.
  type string
ServiceAccount +kind  An identity for processes in pods.
  secrets []ObjectReference
  imagePullSecrets []LocalObjectReference
  automountServiceAccountToken boolean
LimitRange +kind  Per-namespace resource defaults and bounds.
  spec LimitRangeSpec
LimitRangeSpec  Limits of a LimitRange.
  limits []LimitRangeItem!
LimitRangeItem  Bounds for one kind of object.
  type string  Pod, Container or PersistentVolumeClaim.
  max {}quantity
  min {}quantity
  default {}quantity
  defaultRequest {}quantity
  maxLimitRequestRatio {}quantity
ResourceQuota +kind  Aggregate resource limits of a namespace.
  spec ResourceQuotaSpec
  status ResourceQuotaStatus
ResourceQuotaSpec  Hard limits and scopes.
  hard {}quantity
  scopes []string
ResourceQuotaStatus  Enforced and used amounts.
  hard {}quantity
  used {}quantity
ReplicationController +kind  Keeps a number of pod replicas running.
  spec ReplicationControllerSpec
  status ReplicationControllerStatus
ReplicationControllerSpec  Desired replicas.
  replicas integer
  minReadySeconds integer
  selector {}string
  template PodTemplateSpec
ReplicationControllerStatus  Observed replicas.
  replicas integer!
  fullyLabeledReplicas integer
  readyReplicas integer
  availableReplicas integer
  observedGeneration long
  conditions []ReplicationControllerCondition
ReplicationControllerCondition  One condition of a replication controller.
  type string!
  status string!
  lastTransitionTime time
  reason string
  message string
PodTemplate +kind  A stored pod template.
  template PodTemplateSpec
PodTemplateSpec  Metadata and spec of pods to create.
  metadata ObjectMeta
  spec PodSpec

@io.k8s.api.apps.v1
Deployment +kind  Declarative updates for pods and replica sets.
  spec DeploymentSpec
  status DeploymentStatus
DeploymentSpec  Desired state of a deployment.
  replicas integer
  selector LabelSelector!
  template PodTemplateSpec!
  strategy DeploymentStrategy
  minReadySeconds integer
  revisionHistoryLimit integer
  paused boolean
  progressDeadlineSeconds integer
DeploymentRollback +kind  A rollback request (the deployments/rollback subresource).
  name string!
  updatedAnnotations {}string
  rollbackTo io.k8s.api.extensions.v1beta1.RollbackConfig!
DeploymentStrategy  How pods are replaced.
  type string  Recreate or RollingUpdate.
  rollingUpdate RollingUpdateDeployment
RollingUpdateDeployment  Rolling update bounds.
  maxUnavailable ios
  maxSurge ios
DeploymentStatus  Observed state of a deployment.
  observedGeneration long
  replicas integer
  updatedReplicas integer
  readyReplicas integer
  availableReplicas integer
  unavailableReplicas integer
  conditions []DeploymentCondition
  collisionCount integer
DeploymentCondition  One condition of a deployment.
  type string!
  status string!
  lastUpdateTime time
  lastTransitionTime time
  reason string
  message string
DaemonSet +kind  Runs a pod on every eligible node (the AMD device plugin ships as one).
  spec DaemonSetSpec
  status DaemonSetStatus
DaemonSetSpec  Desired state of a daemon set.
  selector LabelSelector!
  template PodTemplateSpec!
  updateStrategy DaemonSetUpdateStrategy
  minReadySeconds integer
  revisionHistoryLimit integer
DaemonSetUpdateStrategy  How daemon pods are replaced.
  type string  OnDelete or RollingUpdate.
  rollingUpdate RollingUpdateDaemonSet
RollingUpdateDaemonSet  Rolling update bound.
  maxUnavailable ios
DaemonSetStatus  Observed state of a daemon set.
  currentNumberScheduled integer!
  numberMisscheduled integer!
  desiredNumberScheduled integer!
  numberReady integer!
  observedGeneration long
  updatedNumberScheduled integer
  numberAvailable integer
  numberUnavailable integer
  collisionCount integer
  conditions []DaemonSetCondition  Latest observations of the daemon set's state.
DaemonSetCondition  One condition of a daemon set.
  type string!
  status string!  True, False or Unknown.
  lastTransitionTime time
  reason string
  message string
ReplicaSet +kind  Keeps a number of pod replicas running.
  spec ReplicaSetSpec
  status ReplicaSetStatus
ReplicaSetSpec  Desired replicas.
  replicas integer
  minReadySeconds integer
  selector LabelSelector!
  template PodTemplateSpec
ReplicaSetStatus  Observed replicas.
  replicas integer!
  fullyLabeledReplicas integer
  readyReplicas integer
  availableReplicas integer
  observedGeneration long
  conditions []ReplicaSetCondition
ReplicaSetCondition  One condition of a replica set.
  type string!
  status string!
  lastTransitionTime time
  reason string
  message string
StatefulSet +kind  Pods with stable identities and storage.
  spec StatefulSetSpec
  status StatefulSetStatus
StatefulSetSpec  Desired state of a stateful set.
  replicas integer
  selector LabelSelector!
  template PodTemplateSpec!
  volumeClaimTemplates []PersistentVolumeClaim
  serviceName string!
  podManagementPolicy string  OrderedReady or Parallel.
  updateStrategy StatefulSetUpdateStrategy
  revisionHistoryLimit integer
StatefulSetUpdateStrategy  How stateful pods are replaced.
  type string  RollingUpdate or OnDelete.
  rollingUpdate RollingUpdateStatefulSetStrategy
RollingUpdateStatefulSetStrategy  Partitioned rolling update.
  partition integer
StatefulSetStatus  Observed state of a stateful set.
  observedGeneration long
  replicas integer!
  readyReplicas integer
  currentReplicas integer
  updatedReplicas integer
  currentRevision string
  updateRevision string
  collisionCount integer
  conditions []StatefulSetCondition  Latest observations of the stateful set's state.
StatefulSetCondition  One condition of a stateful set.
  type string!
  status string!  True, False or Unknown.
  lastTransitionTime time
  reason string
  message string
ControllerRevision +kind  An immutable snapshot of a controller's template.
  data io.k8s.apimachinery.pkg.runtime.RawExtension
  revision long!

@io.k8s.api.apps.v1beta1
Deployment +kind  apps/v1beta1 form of a deployment (stored as apps/v1).
  spec io.k8s.api.extensions.v1beta1.DeploymentSpec
  status io.k8s.api.apps.v1.DeploymentStatus

@io.k8s.api.batch.v1
Job +kind  Runs pods to completion.
  spec JobSpec
  status JobStatus
JobSpec  Desired state of a job.
  parallelism integer
  completions integer
  activeDeadlineSeconds long
  backoffLimit integer
  selector LabelSelector
  manualSelector boolean
  template PodTemplateSpec!
JobStatus  Observed state of a job.
  conditions []JobCondition
  startTime time
  completionTime time
  active integer
  succeeded integer
  failed integer
JobCondition  One condition of a job.
  type string!  Complete or Failed.
  status string!
  lastProbeTime time
  lastTransitionTime time
  reason string
  message string

@io.k8s.api.batch.v1beta1
CronJob +kind  Runs jobs on a schedule.
  spec CronJobSpec
  status CronJobStatus
CronJobSpec  Schedule and job template.
  schedule string!  Cron format.
  startingDeadlineSeconds long
  concurrencyPolicy string  Allow, Forbid or Replace.
  suspend boolean
  jobTemplate JobTemplateSpec!
  successfulJobsHistoryLimit integer
  failedJobsHistoryLimit integer
JobTemplateSpec  Metadata and spec of jobs to create.
  metadata ObjectMeta
  spec io.k8s.api.batch.v1.JobSpec
CronJobStatus  Observed state of a cron job.
  active []ObjectReference
  lastScheduleTime time

@io.k8s.api.coordination.v1
Lease +kind  A lock record (leader election, node heartbeats).
  spec LeaseSpec
LeaseSpec  Holder and timing of a lease.
  holderIdentity string
  leaseDurationSeconds integer
  acquireTime time
  renewTime time
  leaseTransitions integer

@io.k8s.api.scheduling.v1
PriorityClass +kind  Maps a priority class name to a priority value.
  value integer!
  globalDefault boolean
  description string

@io.k8s.api.autoscaling.v1
HorizontalPodAutoscaler +kind  Scales a workload on observed metrics (CPU and MI355X utilisation).
  spec HorizontalPodAutoscalerSpec
  status HorizontalPodAutoscalerStatus
HorizontalPodAutoscalerSpec  Target and bounds.
  scaleTargetRef CrossVersionObjectReference!
  minReplicas integer
  maxReplicas integer!
  targetCPUUtilizationPercentage integer  autoscaling/v1 target.
CrossVersionObjectReference  The scaled object.
  kind string!
  name string!
  apiVersion string
HorizontalPodAutoscalerStatus  Observed state of an autoscaler.
  observedGeneration long
  lastScaleTime time
  currentReplicas integer!
  desiredReplicas integer!
  currentCPUUtilizationPercentage integer
Scale +kind  The scale subresource.
  spec ScaleSpec
  status ScaleStatus
ScaleSpec  Desired replicas.
  replicas integer
ScaleStatus  Observed replicas.
  replicas integer!
  selector string

@io.k8s.api.autoscaling.v2beta1
HorizontalPodAutoscaler +kind  Scales a workload on several metrics (CPU, memory, MI355X utilisation, custom).
  spec HorizontalPodAutoscalerSpec
  status HorizontalPodAutoscalerStatus
HorizontalPodAutoscalerSpec  Target, bounds and metrics.
  scaleTargetRef io.k8s.api.autoscaling.v1.CrossVersionObjectReference!
  minReplicas integer
  maxReplicas integer!
  metrics []MetricSpec  Targets; the largest desired replica count wins.
HorizontalPodAutoscalerStatus  Observed state of an autoscaler.
  observedGeneration long
  lastScaleTime time
  currentReplicas integer!
  desiredReplicas integer!
  currentMetrics []MetricStatus!  Last read value of every metric.
  conditions []HorizontalPodAutoscalerCondition!  Whether the autoscaler can scale, and why.
HorizontalPodAutoscalerCondition  One condition of an autoscaler.
  type string!  ScalingActive, AbleToScale or ScalingLimited.
  status string!
  lastTransitionTime time
  reason string
  message string
MetricStatus  The last read value of one metric.
  type string!  Object, Pods or Resource.
  object ObjectMetricStatus
  pods PodsMetricStatus
  resource ResourceMetricStatus
ObjectMetricStatus  A metric of another object.
  target io.k8s.api.autoscaling.v1.CrossVersionObjectReference!
  metricName string!
  currentValue quantity!
PodsMetricStatus  A per-pod metric averaged over the pods.
  metricName string!
  currentAverageValue quantity!
ResourceMetricStatus  A resource metric averaged over the pods.
  name string!
  currentAverageUtilization integer
  currentAverageValue quantity!
MetricSpec  One autoscaling/v2beta1 metric target.
  type string!  Object, Pods or Resource.
  object ObjectMetricSource
  pods PodsMetricSource
  resource ResourceMetricSource
ObjectMetricSource  A metric of another object.
  target io.k8s.api.autoscaling.v1.CrossVersionObjectReference!
  metricName string!
  targetValue quantity!
PodsMetricSource  A per-pod metric averaged over the pods.
  metricName string!
  targetAverageValue quantity!
ResourceMetricSource  A resource metric (cpu, memory, amd.com/gpu).
  name string!
  targetAverageUtilization integer
  targetAverageValue quantity

@io.k8s.api.policy.v1beta1
PodDisruptionBudget +kind  Bounds voluntary disruptions of a set of pods.
  spec PodDisruptionBudgetSpec
  status PodDisruptionBudgetStatus
PodDisruptionBudgetSpec  The bound.
  minAvailable ios
  selector LabelSelector
  maxUnavailable ios
PodDisruptionBudgetStatus  Observed state of a budget.
  observedGeneration long
  disruptedPods {}time!
  disruptionsAllowed integer!
  currentHealthy integer!
  desiredHealthy integer!
  expectedPods integer!
Eviction +kind  A request to evict a pod, honouring disruption budgets.
  deleteOptions DeleteOptions

@io.k8s.api.extensions.v1beta1
Deployment +kind  extensions/v1beta1 form of a deployment (stored as apps/v1).
  spec DeploymentSpec
  status io.k8s.api.apps.v1.DeploymentStatus
DeploymentSpec  Desired state of a deployment, with the v1beta1 rollback request.
  replicas integer
  selector io.k8s.apimachinery.pkg.apis.meta.v1.LabelSelector
  template io.k8s.api.core.v1.PodTemplateSpec!
  strategy io.k8s.api.apps.v1.DeploymentStrategy
  minReadySeconds integer
  revisionHistoryLimit integer
  paused boolean
  rollbackTo RollbackConfig  The revision to roll back to; cleared by the controller once done.
  progressDeadlineSeconds integer
RollbackConfig  A rollback target.
  revision long  Revision to roll back to; 0 means the previous one.
DaemonSet +kind  extensions/v1beta1 form of a daemon set (stored as apps/v1).
  spec DaemonSetSpec
  status io.k8s.api.apps.v1.DaemonSetStatus
DaemonSetSpec  Desired state of a daemon set, with the v1beta1 template generation.
  selector io.k8s.apimachinery.pkg.apis.meta.v1.LabelSelector
  template io.k8s.api.core.v1.PodTemplateSpec!
  updateStrategy io.k8s.api.apps.v1.DaemonSetUpdateStrategy
  minReadySeconds integer
  templateGeneration long  Generation of the template, kept for the OnDelete history.
  revisionHistoryLimit integer

Ingress +kind  HTTP routing into services.
  spec IngressSpec
  status IngressStatus
IngressSpec  Rules of an ingress.
  backend IngressBackend
  tls []IngressTLS
  rules []IngressRule
IngressBackend  A service port.
  serviceName string!
  servicePort ios!
IngressTLS  TLS for a set of hosts.
  hosts []string
  secretName string
IngressRule  Routing for one host.
  host string
  http HTTPIngressRuleValue
HTTPIngressRuleValue  Paths of a host.
  paths []HTTPIngressPath!
HTTPIngressPath  One path.
  path string
  backend IngressBackend!
IngressStatus  Observed state of an ingress.
  loadBalancer LoadBalancerStatus
PodSecurityPolicy +kind  Cluster-wide pod security rules.
  spec PodSecurityPolicySpec
PodSecurityPolicySpec  The rules.
  privileged boolean
  defaultAddCapabilities []string
  requiredDropCapabilities []string
  allowedCapabilities []string
  volumes []string
  hostNetwork boolean
  hostPorts []HostPortRange
  hostPID boolean
  hostIPC boolean
  seLinux SELinuxStrategyOptions!
  runAsUser RunAsUserStrategyOptions!
  supplementalGroups SupplementalGroupsStrategyOptions!
  fsGroup FSGroupStrategyOptions!
  readOnlyRootFilesystem boolean
  defaultAllowPrivilegeEscalation boolean
  allowPrivilegeEscalation boolean
  allowedHostPaths []AllowedHostPath
  allowedFlexVolumes []AllowedFlexVolume  Flexvolume drivers pods may use; empty allows all (when "flexVolume" is in volumes).
AllowedFlexVolume  A Flexvolume driver pods may use.
  driver string!  Name of the driver.
HostPortRange  Allowed host ports.
  min integer!
  max integer!
SELinuxStrategyOptions  SELinux strategy.
  rule string!
  seLinuxOptions SELinuxOptions
RunAsUserStrategyOptions  User strategy.
  rule string!
  ranges []IDRange
SupplementalGroupsStrategyOptions  Supplemental group strategy.
  rule string
  ranges []IDRange
FSGroupStrategyOptions  fsGroup strategy.
  rule string
  ranges []IDRange
IDRange  An ID range.
  min long!
  max long!
AllowedHostPath  An allowed hostPath prefix.
  pathPrefix string

@io.k8s.api.networking.v1
NetworkPolicy +kind  Allowed traffic for a set of pods.
  spec NetworkPolicySpec
NetworkPolicySpec  Selected pods and rules.
  podSelector LabelSelector!
  ingress []NetworkPolicyIngressRule
  egress []NetworkPolicyEgressRule
  policyTypes []string
NetworkPolicyIngressRule  Allowed inbound traffic.
  ports []NetworkPolicyPort
  from []NetworkPolicyPeer
NetworkPolicyEgressRule  Allowed outbound traffic.
  ports []NetworkPolicyPort
  to []NetworkPolicyPeer
NetworkPolicyPort  A port.
  protocol string
  port ios
NetworkPolicyPeer  A peer.
  podSelector LabelSelector
  namespaceSelector LabelSelector
  ipBlock IPBlock
IPBlock  A CIDR with exceptions.
  cidr string!
  except []string

@io.k8s.api.settings.v1alpha1
PodPreset +kind  Injects settings into matching pods at admission.
  spec PodPresetSpec
PodPresetSpec  What is injected.
  selector LabelSelector
  env []EnvVar
  envFrom []EnvFromSource
  volumes []Volume
  volumeMounts []VolumeMount

@io.k8s.api.certificates.v1beta1
CertificateSigningRequest +kind  A request for a signed certificate.
  spec CertificateSigningRequestSpec
  status CertificateSigningRequestStatus
CertificateSigningRequestSpec  The request.
  request byte!  PEM PKCS#10 request.
  usages []string
  username string
  uid string
  groups []string
  extra {}[]string
CertificateSigningRequestStatus  Approval and the issued certificate.
  conditions []CertificateSigningRequestCondition
  certificate byte
CertificateSigningRequestCondition  Approved or Denied.
  type string!
  reason string
  message string
  lastUpdateTime time

@io.k8s.api.rbac.v1
Role +kind  Namespaced permissions.
  rules []PolicyRule!
ClusterRole +kind  Cluster-wide permissions.
  rules []PolicyRule!  Empty for an aggregated role: the controller fills it from the selected roles.
  aggregationRule AggregationRule
AggregationRule  Selects cluster roles whose rules are aggregated.
  clusterRoleSelectors []LabelSelector
PolicyRule  Allowed verbs on resources or URLs.
  verbs []string!
  apiGroups []string
  resources []string
  resourceNames []string
  nonResourceURLs []string
RoleBinding +kind  Grants a role within a namespace.
  subjects []Subject!
  roleRef RoleRef!
ClusterRoleBinding +kind  Grants a cluster role everywhere.
  subjects []Subject!
  roleRef RoleRef!
Subject  A user, group or service account.
  kind string!
  apiGroup string
  name string!
  namespace string
RoleRef  The granted role.
  apiGroup string!
  kind string!
  name string!

@io.k8s.api.storage.v1
StorageClass +kind  A class of dynamically provisioned storage.
  provisioner string!
  parameters {}string
  reclaimPolicy string
  mountOptions []string
  allowVolumeExpansion boolean
  volumeBindingMode string  Immediate or WaitForFirstConsumer.

@io.k8s.api.storage.v1beta1
VolumeAttachment +kind  Intent to attach a volume to a node (CSI).
  spec VolumeAttachmentSpec!
  status VolumeAttachmentStatus
VolumeAttachmentSpec  What to attach where.
  attacher string!
  source VolumeAttachmentSource!
  nodeName string!
VolumeAttachmentSource  The volume.
  persistentVolumeName string
VolumeAttachmentStatus  Attach state.
  attached boolean!
  attachmentMetadata {}string
  attachError VolumeError
  detachError VolumeError
VolumeError  An attach or detach error.
  time time
  message string

@io.k8s.api.authorization.v1
SubjectAccessReview +kind  Asks whether a user may perform an action.
  spec SubjectAccessReviewSpec!
  status SubjectAccessReviewStatus
SelfSubjectAccessReview +kind  Asks whether the caller may perform an action.
  spec SelfSubjectAccessReviewSpec!
  status SubjectAccessReviewStatus
LocalSubjectAccessReview +kind  A namespaced SubjectAccessReview.
  spec SubjectAccessReviewSpec!
  status SubjectAccessReviewStatus
SubjectAccessReviewSpec  The action and the user.
  resourceAttributes ResourceAttributes
  nonResourceAttributes NonResourceAttributes
  user string
  groups []string
  extra {}[]string
  uid string
SelfSubjectAccessReviewSpec  The action.
  resourceAttributes ResourceAttributes
  nonResourceAttributes NonResourceAttributes
ResourceAttributes  A resource request.
  namespace string
  verb string
  group string
  version string
  resource string
  subresource string
  name string
NonResourceAttributes  A non-resource request.
  path string
  verb string
SubjectAccessReviewStatus  The answer.
  allowed boolean!
  denied boolean
  reason string
  evaluationError string

@io.k8s.api.authentication.v1
TokenReview +kind  Asks who a bearer token belongs to.
  spec TokenReviewSpec!
  status TokenReviewStatus
TokenReviewSpec  The token.
  token string
TokenReviewStatus  The answer.
  authenticated boolean
  user UserInfo
  error string
UserInfo  An authenticated user.
  username string
  uid string
  groups []string
  extra {}[]string

@io.k8s.api.admissionregistration.v1beta1
MutatingWebhookConfiguration +kind  Webhooks that may change objects at admission.
  webhooks []Webhook
ValidatingWebhookConfiguration +kind  Webhooks that may reject objects at admission.
  webhooks []Webhook
Webhook  One admission webhook.
  name string!
  clientConfig WebhookClientConfig!
  rules []RuleWithOperations
  failurePolicy string  Ignore or Fail.
  namespaceSelector LabelSelector
WebhookClientConfig  How to reach a webhook.
  url string
  service ServiceReference
  caBundle byte!
ServiceReference  An in-cluster webhook service.
  namespace string!
  name string!
  path string
RuleWithOperations  Operations and resources a webhook sees.
  operations []string
  apiGroups []string
  apiVersions []string
  resources []string

@io.k8s.api.admissionregistration.v1alpha1
InitializerConfiguration +kind  Initializers added to new objects.
  initializers []Initializer
Initializer  One initializer and the resources it applies to.
  name string!
  rules []Rule
Rule  Groups, versions and resources.
  apiGroups []string
  apiVersions []string
  resources []string

@io.k8s.apiextensions-apiserver.pkg.apis.apiextensions.v1beta1
CustomResourceDefinition +kind  Adds a resource served by the API server.
  spec CustomResourceDefinitionSpec
  status CustomResourceDefinitionStatus
CustomResourceDefinitionSpec  Group, names and schema.
  group string!
  version string!
  names CustomResourceDefinitionNames!
  scope string!  Namespaced or Cluster.
  validation CustomResourceValidation
  subresources object
CustomResourceDefinitionNames  Names of a custom resource.
  plural string!
  singular string
  shortNames []string
  kind string!
  listKind string
  categories []string
CustomResourceValidation  Validation schema.
  openAPIV3Schema JSONSchemaProps
JSONSchemaProps  A JSON-Schema (draft 4, OpenAPI v3 subset) document; free-form below this point.
  id string
  $schema string
  $ref string
  description string
  type string
  format string
  title string
  default JSON
  maximum number
  exclusiveMaximum boolean
  minimum number
  exclusiveMinimum boolean
  maxLength long
  minLength long
  pattern string
  maxItems long
  minItems long
  uniqueItems boolean
  multipleOf number
  enum []JSON
  maxProperties long
  minProperties long
  required []string
  items JSONSchemaPropsOrArray
  allOf []JSONSchemaProps
  oneOf []JSONSchemaProps
  anyOf []JSONSchemaProps
  not JSONSchemaProps
  properties {}JSONSchemaProps
  additionalProperties JSONSchemaPropsOrBool
  patternProperties {}JSONSchemaProps
  dependencies {}JSONSchemaPropsOrStringArray
  additionalItems JSONSchemaPropsOrBool
  definitions {}JSONSchemaProps
  externalDocs ExternalDocumentation
  example JSON
JSON  Any JSON value.
  Raw byte!
JSONSchemaPropsOrArray  A schema or an array of schemas.
  Schema JSONSchemaProps!
  JSONSchemas []JSONSchemaProps!
JSONSchemaPropsOrBool  A schema or a boolean.
  Allows boolean!
  Schema JSONSchemaProps!
JSONSchemaPropsOrStringArray  A schema or a list of property names.
  Schema JSONSchemaProps!
  Property []string!
ExternalDocumentation  A link to more documentation.
  description string
  url string
CustomResourceDefinitionCondition  One condition of a definition.
  type string!  Established or NamesAccepted.
  status string!
  lastTransitionTime time
  reason string
  message string
CustomResourceDefinitionStatus  Observed state of a definition.
  conditions []CustomResourceDefinitionCondition!
  acceptedNames CustomResourceDefinitionNames!

@io.k8s.kube-aggregator.pkg.apis.apiregistration.v1beta1
APIService +kind  A group version served by another server through the aggregator.
  spec APIServiceSpec
  status APIServiceStatus
APIServiceSpec  Where the group version is served.
  service ServiceReference!
  group string
  version string
  insecureSkipTLSVerify boolean
  caBundle byte!
  groupPriorityMinimum integer!
  versionPriority integer!
ServiceReference  The serving service.
  namespace string
  name string
APIServiceStatus  Availability.
  conditions []APIServiceCondition
APIServiceCondition  One condition of an API service.
  type string!  Available.
  status string!
  lastTransitionTime time
  reason string
  message string

@io.k8s.apimachinery.pkg.runtime
RawExtension  An embedded object of any kind, carried as its own serialized bytes.
  Raw byte!  The object's bytes (JSON or protobuf).
"""

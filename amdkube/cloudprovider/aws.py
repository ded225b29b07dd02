"""The AWS cloud provider: EC2 instances/zones/routes, classic ELB load balancers, EBS volumes.

The fork's README lists EC2 GPU VMs among its supported platforms; this is the
same provider for GPU instances on AWS. Reference: pkg/cloudprovider/providers/aws —
  * aws.go NodeAddresses / extractNodeAddresses (every in-use ENI's private IPs are InternalIP,
    the public IP ExternalIP, private/public DNS names InternalDNS/ExternalDNS; the node name is
    the private DNS name), InstanceID `/<az>/<instance-id>` (providerID `aws:///<az>/<id>`),
    InstanceType, GetZone* (the availability zone; the region is the zone minus its letter);
  * tags.go: cluster ownership by `kubernetes.io/cluster/<id>` (owned|shared) or the legacy
    `KubernetesCluster=<id>` tag;
  * aws_routes.go: one route table (RouteTableID or the cluster-tagged one); a route per node
    CIDR with the instance as target after source/dest check is disabled; blackhole routes for
    the same CIDR are replaced; route name `<cluster>-<cidr>`;
  * aws.go EnsureLoadBalancer / aws_loadbalancer.go: a classic ELB named after the service UID
    (`a` + uid without dashes, 32 chars), one TCP/SSL listener per port to its nodePort, the
    cluster's subnets (one per zone, `kubernetes.io/role/elb` or `.../internal-elb` preferred),
    a `k8s-elb-<name>` security group opened to loadBalancerSourceRanges, node security groups
    opened to it, a TCP (or HTTP for externalTrafficPolicy=Local) health check, attributes and
    health-check thresholds from the service.beta.kubernetes.io/aws-load-balancer-* annotations;
  * aws.go Create/Delete/Attach/DetachDisk, device_allocator.go (devices /dev/xvdba…/dev/xvdcz
    handed out least-recently-used first), volumes.go (volume IDs `aws://<az>/vol-…`).

The EC2 (2016-11-15) and ELB (2012-06-01) query APIs are spoken directly — Signature V4, form
POST, XML answers — with `requests`; credentials come from the config, the environment or the
instance's IAM role through the metadata service. On Nitro GPU instances EBS disks appear as
NVMe namespaces, so the kubelet also looks for /dev/disk/by-id/nvme-Amazon_Elastic_Block_Store_vol…
"""
from __future__ import annotations

import configparser
import datetime
import hashlib
import hmac
import json
import logging
import os
import re
import threading
import time
import xml.etree.ElementTree as ET
from urllib.parse import quote, urlsplit

from . import Interface, Route, Zone, off_loop
from ..api import meta as m

log = logging.getLogger("amdkube.cloudprovider.aws")
PROVIDER = "aws"
METADATA_URL = "http://169.254.169.254/latest/meta-data/"
EC2_VERSION, ELB_VERSION = "2016-11-15", "2012-06-01"
TAG_CLUSTER_LEGACY = "KubernetesCluster"
TAG_CLUSTER_PREFIX = "kubernetes.io/cluster/"
TAG_SERVICE = "kubernetes.io/service-name"
TAG_ELB_PUBLIC, TAG_ELB_INTERNAL = "kubernetes.io/role/elb", "kubernetes.io/role/internal-elb"
ANN = "service.beta.kubernetes.io/aws-load-balancer-"
EBS_PROVISIONER = "kubernetes.io/aws-ebs"
DEFAULT_VOLUME_TYPE = "gp2"


class AWSError(RuntimeError):
    def __init__(self, status: int, code: str, msg: str):
        super().__init__(f"aws: {code} (HTTP {status}): {msg}")
        self.status, self.code = status, code


# ----------------------------------------------------------------------------- Signature V4
def _hmac(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def sign_v4(method: str, url: str, headers: dict, body: bytes, region: str, service: str,
            access_key: str, secret_key: str, amz_date: str, session_token: str = "") -> dict:
    """AWS Signature Version 4 (the algorithm of the public SigV4 test suite): returns the
    headers to send, Authorization included. `headers` must not hold Authorization."""
    u = urlsplit(url)
    hdrs = {k.lower(): " ".join(str(v).split()) for k, v in headers.items()}
    hdrs.setdefault("host", u.netloc)
    hdrs["x-amz-date"] = amz_date
    if session_token:
        hdrs["x-amz-security-token"] = session_token
    signed = ";".join(sorted(hdrs))
    canon_headers = "".join(f"{k}:{hdrs[k]}\n" for k in sorted(hdrs))
    pairs = []
    for part in u.query.split("&") if u.query else []:
        k, _, v = part.partition("=")
        pairs.append((quote(_unquote(k), safe="-_.~"), quote(_unquote(v), safe="-_.~")))
    canon_query = "&".join(f"{k}={v}" for k, v in sorted(pairs))
    path = quote(u.path or "/", safe="/-_.~")
    creq = "\n".join([method, path, canon_query, canon_headers, signed, hashlib.sha256(body).hexdigest()])
    day = amz_date[:8]
    scope = f"{day}/{region}/{service}/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(creq.encode()).hexdigest()])
    k = _hmac(_hmac(_hmac(_hmac(("AWS4" + secret_key).encode(), day), region), service), "aws4_request")
    sig = hmac.new(k, sts.encode(), hashlib.sha256).hexdigest()
    out = {k2: v for k2, v in hdrs.items() if k2 != "host"}
    out["Authorization"] = f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, SignedHeaders={signed}, Signature={sig}"
    return out


def _unquote(s: str) -> str:
    from urllib.parse import unquote_plus
    return unquote_plus(s)


# ----------------------------------------------------------------------------- XML ⇄ python
def xml_to_obj(el):
    """An EC2/ELB answer element → python: `item`/`member` children make lists, leaves are text."""
    kids = list(el)
    if not kids:
        return el.text or ""
    tags = [_local(k.tag) for k in kids]
    if all(t in ("item", "member") for t in tags):
        return [xml_to_obj(k) for k in kids]
    return {t: xml_to_obj(k) for t, k in zip(tags, kids)}


def _local(tag: str) -> str:
    return tag.rsplit("}", 1)[-1]


def _list(v) -> list:
    """An EC2 set that may be empty ('' from an empty element) or a single-item list."""
    if isinstance(v, list):
        return v
    return [] if v in ("", None) else [v]


def ec2_params(prefix: str, items, style: str = "ec2") -> dict:
    """Flatten a list (of scalars or dicts) into query parameters: EC2 `Name.N[.Key]`,
    ELB `Name.member.N[.Key]`; nested lists recurse with the same style."""
    out = {}
    for i, it in enumerate(items, 1):
        base = f"{prefix}.member.{i}" if style == "elb" else f"{prefix}.{i}"
        if isinstance(it, dict):
            for k, v in it.items():
                if isinstance(v, list):
                    out.update(ec2_params(f"{base}.{k}", v, style))
                elif isinstance(v, dict):
                    for k2, v2 in v.items():
                        out[f"{base}.{k}.{k2}"] = _s(v2)
                elif v is not None:
                    out[f"{base}.{k}"] = _s(v)
        else:
            out[base] = _s(it)
    return out


def _s(v) -> str:
    return ("true" if v else "false") if isinstance(v, bool) else str(v)


def tags_of(obj: dict) -> dict:
    return {t.get("key", t.get("Key", "")): t.get("value", t.get("Value", "")) for t in _list(obj.get("tagSet") or obj.get("Tags"))}


# ----------------------------------------------------------------------------- config
def parse_config(cfg) -> dict:
    """aws.conf ([Global] gcfg keys, case-insensitive) or a dict → {lower-key: value}."""
    if isinstance(cfg, str):
        try:
            cfg = json.loads(cfg)
        except ValueError:
            cp = configparser.ConfigParser(interpolation=None)
            cp.read_string(cfg)
            cfg = {s: dict(cp.items(s)) for s in cp.sections()}
    cfg = cfg or {}
    glob = next((v for k, v in cfg.items() if str(k).lower() == "global"), None)
    flat = glob if isinstance(glob, dict) else cfg
    out = {str(k).lower(): v for k, v in flat.items() if not isinstance(v, dict)}
    for k, v in cfg.items():
        if isinstance(v, dict) and str(k).lower() != "global":
            out[str(k).lower()] = {str(k2).lower(): v2 for k2, v2 in v.items()}
    return out


def _truthy(v) -> bool:
    return str(v).strip().lower() in ("1", "true", "yes")


# ----------------------------------------------------------------------------- metadata + client
class Metadata:
    """The EC2 instance metadata service (ec2metadata): plain-text paths under meta-data/."""

    def __init__(self, http, url: str = METADATA_URL):
        self.http, self.url = http, url.rstrip("/") + "/"

    def get(self, path: str) -> str:
        r = self.http.get(self.url + path.lstrip("/"), timeout=5)
        if r.status_code != 200:
            raise AWSError(r.status_code, "MetadataError", f"{path}: {r.text[:120]}")
        return r.text


class Client:
    """Signed EC2 / ELB query calls with credentials from config, environment or the IAM role."""

    def __init__(self, cfg: dict, metadata: Metadata, http):
        self.cfg, self.md, self.http = cfg, metadata, http
        self.region = ""
        self.endpoints = {"ec2": cfg.get("ec2-endpoint", ""), "elasticloadbalancing": cfg.get("elb-endpoint", "")}
        self._creds = None
        self._lock = threading.Lock()

    def creds(self) -> tuple[str, str, str]:
        with self._lock:
            if self._creds and (self._creds[3] == 0 or self._creds[3] - time.time() > 300):
                return self._creds[:3]
            ak = self.cfg.get("access-key-id") or os.environ.get("AWS_ACCESS_KEY_ID", "")
            sk = self.cfg.get("secret-access-key") or os.environ.get("AWS_SECRET_ACCESS_KEY", "")
            tok = self.cfg.get("session-token") or os.environ.get("AWS_SESSION_TOKEN", "")
            exp = 0.0
            if not (ak and sk):
                role = self.md.get("iam/security-credentials/").split("\n")[0].strip()
                doc = json.loads(self.md.get(f"iam/security-credentials/{role}"))
                ak, sk, tok = doc["AccessKeyId"], doc["SecretAccessKey"], doc.get("Token", "")
                exp = datetime.datetime.strptime(doc["Expiration"], "%Y-%m-%dT%H:%M:%SZ").replace(
                    tzinfo=datetime.timezone.utc).timestamp() if doc.get("Expiration") else 0.0
            self._creds = (ak, sk, tok, exp)
            return ak, sk, tok

    def call(self, service: str, action: str, params: dict | None = None) -> dict:
        url = self.endpoints.get(service) or f"https://{service}.{self.region}.amazonaws.com/"
        if not url.endswith("/"):
            url += "/"
        form = {"Action": action, "Version": EC2_VERSION if service == "ec2" else ELB_VERSION, **(params or {})}
        body = "&".join(f"{quote(k, safe='-_.~')}={quote(str(v), safe='-_.~')}" for k, v in sorted(form.items())).encode()
        ak, sk, tok = self.creds()
        amz = datetime.datetime.now(datetime.timezone.utc).strftime("%Y%m%dT%H%M%SZ")
        hdrs = sign_v4("POST", url, {"Content-Type": "application/x-www-form-urlencoded; charset=utf-8"}, body,
                       self.region, service, ak, sk, amz, tok)
        r = self.http.post(url, data=body, headers=hdrs, timeout=60)
        try:
            root = ET.fromstring(r.content) if r.content else None
        except ET.ParseError:
            root = None
        if r.status_code >= 400 or root is None:
            code, msg = "Unknown", r.text[:300]
            if root is not None:
                err = next((e for e in root.iter() if _local(e.tag) == "Error"), None)
                if err is not None:
                    d = xml_to_obj(err)
                    code, msg = d.get("Code", code), d.get("Message", msg)
            raise AWSError(r.status_code, code, f"{action}: {msg}")
        out = xml_to_obj(root)
        if service != "ec2" and isinstance(out, dict):       # ELB wraps answers in <ActionResult>
            out = out.get(f"{action}Result", out)
        return out if isinstance(out, dict) else {}


# ----------------------------------------------------------------------------- instances
def node_addresses(inst: dict) -> list[dict]:
    out = []
    for ni in _list(inst.get("networkInterfaceSet")):
        if ni.get("status", "in-use") != "in-use":
            continue
        for pa in _list(ni.get("privateIpAddressesSet")):
            if pa.get("privateIpAddress"):
                out.append({"type": "InternalIP", "address": pa["privateIpAddress"]})
    if not out and inst.get("privateIpAddress"):
        out.append({"type": "InternalIP", "address": inst["privateIpAddress"]})
    if inst.get("ipAddress"):
        out.append({"type": "ExternalIP", "address": inst["ipAddress"]})
    if inst.get("privateDnsName"):
        out.append({"type": "InternalDNS", "address": inst["privateDnsName"]})
    if inst.get("dnsName"):
        out.append({"type": "ExternalDNS", "address": inst["dnsName"]})
    return out


def instance_id_from_provider_id(pid: str) -> str:
    """`aws:///<az>/<id>`, `aws://<az>/<id>`, `/<az>/<id>` or a bare `i-…` → `i-…`."""
    s = pid[len("aws://"):] if pid.startswith("aws://") else pid
    iid = s.rstrip("/").rsplit("/", 1)[-1]
    if not re.fullmatch(r"i-[a-z0-9]+", iid):
        raise ValueError(f"invalid AWS instance id in {pid!r}")
    return iid


def _az(inst: dict) -> str:
    return (inst.get("placement") or {}).get("availabilityZone", "")


class Instances:
    def __init__(self, aws):
        self.aws = aws

    def describe(self, filters: list[dict] | None = None, ids: list[str] | None = None) -> list[dict]:
        params = {}
        if filters:
            params.update(ec2_params("Filter", [{"Name": f["Name"], "Value": f["Values"]} for f in filters]))
        if ids:
            params.update(ec2_params("InstanceId", ids))
        out = []
        for res in _list(self.aws.client.call("ec2", "DescribeInstances", params).get("reservationSet")):
            out.extend(_list(res.get("instancesSet")))
        return out

    def by_name(self, name: str) -> dict:
        """mapNodeNameToPrivateDNSName: nodes are named by their private DNS name."""
        got = [i for i in self.describe([{"Name": "private-dns-name", "Values": [name]}])
               if (i.get("instanceState") or {}).get("name") not in ("terminated", "shutting-down")]
        if not got:
            raise LookupError(f"instance not found: {name}")
        if len(got) > 1:
            raise LookupError(f"multiple instances found for name: {name}")
        return got[0]

    def by_id(self, iid: str) -> dict | None:
        try:
            got = self.describe(ids=[iid])
        except AWSError as e:
            if e.code == "InvalidInstanceID.NotFound":
                return None
            raise
        return got[0] if got else None

    @off_loop
    def node_addresses(self, name: str) -> list[dict]:
        return node_addresses(self.by_name(name))

    @off_loop
    def node_addresses_by_provider_id(self, pid: str) -> list[dict]:
        inst = self.by_id(instance_id_from_provider_id(pid))
        if inst is None:
            raise LookupError(f"instance not found: {pid}")
        return node_addresses(inst)

    @off_loop
    def instance_exists(self, name: str) -> bool:
        try:
            self.by_name(name)
            return True
        except LookupError:
            return False

    @off_loop
    def instance_exists_by_provider_id(self, pid: str) -> bool:
        inst = self.by_id(instance_id_from_provider_id(pid))
        return inst is not None and (inst.get("instanceState") or {}).get("name") != "terminated"

    @off_loop
    def instance_id(self, name: str) -> str:
        inst = self.by_name(name)
        return f"/{_az(inst)}/{inst['instanceId']}"

    def provider_id_of(self, name: str) -> str:
        inst = self.by_name(name)
        return f"aws:///{_az(inst)}/{inst['instanceId']}"

    @off_loop
    def instance_type(self, name: str) -> str:
        return self.by_name(name).get("instanceType", "")


# ----------------------------------------------------------------------------- tagging
class Tagging:
    """tags.go: which resources belong to this cluster."""

    def __init__(self, cluster_id: str):
        self.cluster_id = cluster_id

    def owns(self, tags: dict) -> bool:
        if not self.cluster_id:
            return True
        return tags.get(TAG_CLUSTER_LEGACY) == self.cluster_id or (TAG_CLUSTER_PREFIX + self.cluster_id) in tags

    def tags(self, extra: dict | None = None) -> dict:
        out = dict(extra or {})
        if self.cluster_id:
            out[TAG_CLUSTER_PREFIX + self.cluster_id] = "owned"
        return out

    def filters(self) -> list[dict]:
        return [{"Name": "tag-key", "Values": [TAG_CLUSTER_PREFIX + self.cluster_id]}] if self.cluster_id else []


def _tag_params(tags: dict, prefix="Tag") -> dict:
    return ec2_params(prefix, [{"Key": k, "Value": v} for k, v in sorted(tags.items())])


# ----------------------------------------------------------------------------- routes
class Routes:
    def __init__(self, aws):
        self.aws = aws

    def _table(self, cluster: str) -> dict:
        c = self.aws.client
        rtid = self.aws.cfg.get("routetableid", "")
        if rtid:
            tables = _list(c.call("ec2", "DescribeRouteTables", ec2_params("Filter", [{"Name": "route-table-id", "Value": [rtid]}]))
                           .get("routeTableSet"))
        else:
            tables = [t for t in _list(c.call("ec2", "DescribeRouteTables", ec2_params(
                "Filter", [{"Name": f["Name"], "Value": f["Values"]} for f in self.aws.tagging.filters()])).get("routeTableSet"))
                if self.aws.tagging.owns(tags_of(t))]
        if not tables:
            raise LookupError(f"unable to find route table for AWS cluster: {cluster}")
        if len(tables) > 1:
            raise LookupError(f"found multiple matching AWS route tables for AWS cluster: {cluster}")
        return tables[0]

    def list(self, cluster: str) -> list[Route]:
        t = self._table(cluster)
        rs = _list(t.get("routeSet"))
        ids = sorted({r["instanceId"] for r in rs if r.get("instanceId") and r.get("state") != "blackhole"})
        # an instance-id filter (not InstanceId.N): a terminated instance is just absent, not an error
        by_id = {i["instanceId"]: i for i in (self.aws.instances_.describe([{"Name": "instance-id", "Values": ids}]) if ids else [])}
        out = []
        for r in rs:
            cidr = r.get("destinationCidrBlock")
            if not cidr:
                continue
            if r.get("state") == "blackhole":
                out.append(Route(f"{cluster}-{cidr}", "", cidr))
                continue
            inst = by_id.get(r.get("instanceId", ""))
            if inst is not None:
                out.append(Route(f"{cluster}-{cidr}", inst.get("privateDnsName", ""), cidr))
        return out

    def create(self, cluster: str, name_hint: str, route: Route):
        c = self.aws.client
        inst = self.aws.instances_.by_name(route.target_node)
        c.call("ec2", "ModifyInstanceAttribute", {"InstanceId": inst["instanceId"], "SourceDestCheck.Value": "false"})
        t = self._table(cluster)
        for r in _list(t.get("routeSet")):
            if r.get("destinationCidrBlock") == route.destination_cidr:
                if r.get("state") == "blackhole" or r.get("instanceId") != inst["instanceId"]:
                    c.call("ec2", "DeleteRoute", {"RouteTableId": t["routeTableId"], "DestinationCidrBlock": route.destination_cidr})
                else:
                    return
        c.call("ec2", "CreateRoute", {"RouteTableId": t["routeTableId"], "DestinationCidrBlock": route.destination_cidr,
                                      "InstanceId": inst["instanceId"]})

    def delete(self, cluster: str, route: Route):
        t = self._table(cluster)
        try:
            self.aws.client.call("ec2", "DeleteRoute", {"RouteTableId": t["routeTableId"],
                                                        "DestinationCidrBlock": route.destination_cidr})
        except AWSError as e:
            if e.code != "InvalidRoute.NotFound":
                raise


# ----------------------------------------------------------------------------- ELB
def lb_name(svc: dict) -> str:
    """cloudprovider.GetLoadBalancerName: "a" + the UID without dashes, at most 32 characters."""
    return ("a" + m.uid_of(svc).replace("-", ""))[:32]


def _ann_int(ann: dict, key: str, default: int) -> int:
    v = ann.get(ANN + key)
    if v is None or v == "":
        return default
    try:
        return int(v)
    except ValueError:
        raise ValueError(f"error parsing service annotation: {ANN + key}={v}") from None


def _ann_bool(ann: dict, key: str, default: bool) -> bool:
    v = ann.get(ANN + key)
    if v is None or v == "":
        return default
    if str(v).lower() not in ("true", "false", "1", "0"):
        raise ValueError(f"error parsing service annotation: {ANN + key}={v}")
    return _truthy(v)


def listeners_for(svc: dict) -> list[dict]:
    """buildListener: TCP by default; SSL/HTTPS on the aws-load-balancer-ssl-ports (all ports
    when unset) when an aws-load-balancer-ssl-cert is given; backend protocol by annotation."""
    ann, spec = m.annotations_of(svc), svc.get("spec") or {}
    cert = ann.get(ANN + "ssl-cert", "")
    ssl_ports = {p.strip() for p in ann.get(ANN + "ssl-ports", "*").split(",") if p.strip()}
    be = ann.get(ANN + "backend-protocol", "").lower()
    out = []
    for p in spec.get("ports") or []:
        if p.get("protocol", "TCP") != "TCP":
            raise ValueError("Only TCP LoadBalancer is supported for AWS ELB")
        if not p.get("nodePort"):
            continue
        proto, iproto = "tcp", "tcp"
        want_ssl = cert and ("*" in ssl_ports or str(p["port"]) in ssl_ports or p.get("name", "") in ssl_ports)
        if be in ("http", "https"):
            iproto = be
            proto = "https" if want_ssl else "http"
        elif be == "ssl":
            iproto, proto = "ssl", "ssl" if want_ssl else "tcp"
        elif want_ssl:
            proto = "ssl"
        lst = {"Protocol": proto.upper(), "LoadBalancerPort": int(p["port"]), "InstanceProtocol": iproto.upper(),
               "InstancePort": int(p["nodePort"])}
        if want_ssl:
            lst["SSLCertificateId"] = cert
        out.append(lst)
    return out


class LoadBalancer:
    def __init__(self, aws):
        self.aws = aws

    # ---- lookups
    def _describe(self, name: str) -> dict | None:
        try:
            d = self.aws.client.call("elasticloadbalancing", "DescribeLoadBalancers", ec2_params("LoadBalancerNames", [name], "elb"))
        except AWSError as e:
            if e.code == "LoadBalancerNotFound":
                return None
            raise
        lbs = _list(d.get("LoadBalancerDescriptions"))
        return lbs[0] if lbs else None

    def get(self, cluster: str, svc: dict):
        lb = self._describe(lb_name(svc))
        return ({"ingress": [{"hostname": lb.get("DNSName", "")}]}, True) if lb else (None, False)

    def _subnets(self, internal: bool) -> list[str]:
        """findELBSubnets: the configured subnet, else the cluster's subnets in the VPC, one per
        zone, preferring the ELB role tag."""
        cfg, c = self.aws.cfg, self.aws.client
        flt = [{"Name": "vpc-id", "Value": [self.aws.vpc_id()]}] if self.aws.vpc_id() else []
        subs = [s for s in _list(c.call("ec2", "DescribeSubnets", ec2_params("Filter", flt)).get("subnetSet"))
                if self.aws.tagging.owns(tags_of(s)) or s.get("subnetId") == cfg.get("subnetid")]
        role = TAG_ELB_INTERNAL if internal else TAG_ELB_PUBLIC
        best: dict[str, dict] = {}
        for s in sorted(subs, key=lambda s: s.get("subnetId", "")):
            az = s.get("availabilityZone", "")
            cur = best.get(az)
            if cur is None or (role in tags_of(s) and role not in tags_of(cur)):
                best[az] = s
        return sorted(s["subnetId"] for s in best.values())

    def _security_group(self, name: str, svc: dict) -> str:
        c, cfg = self.aws.client, self.aws.cfg
        if cfg.get("elbsecuritygroup"):
            return cfg["elbsecuritygroup"]
        gname = f"k8s-elb-{name}"
        flt = [{"Name": "group-name", "Value": [gname]}] + ([{"Name": "vpc-id", "Value": [self.aws.vpc_id()]}] if self.aws.vpc_id() else [])
        got = _list(c.call("ec2", "DescribeSecurityGroups", ec2_params("Filter", flt)).get("securityGroupInfo"))
        if got:
            return got[0]["groupId"]
        params = {"GroupName": gname, "GroupDescription": f"Security group for Kubernetes ELB {name} ({m.key_of(svc)})"}
        if self.aws.vpc_id():
            params["VpcId"] = self.aws.vpc_id()
        gid = c.call("ec2", "CreateSecurityGroup", params)["groupId"]
        c.call("ec2", "CreateTags", {**ec2_params("ResourceId", [gid]), **_tag_params(self.aws.tagging.tags())})
        return gid

    def _set_ingress(self, gid: str, want: list[dict]):
        """setSecurityGroupIngress: make the group's ingress exactly `want`."""
        c = self.aws.client
        grp = _list(c.call("ec2", "DescribeSecurityGroups", ec2_params("GroupId", [gid])).get("securityGroupInfo"))
        have = []
        for p in _list((grp[0] if grp else {}).get("ipPermissions")):
            for r in _list(p.get("ipRanges")):
                have.append((p.get("ipProtocol"), int(p.get("fromPort", 0) or 0), int(p.get("toPort", 0) or 0), r.get("cidrIp")))
        want_t = {(w["IpProtocol"], w["FromPort"], w["ToPort"], cidr) for w in want for cidr in w["Cidrs"]}
        add = sorted(want_t - set(have))
        rm = sorted(set(have) - want_t)

        def perms(rules):
            return ec2_params("IpPermissions", [{"IpProtocol": p, "FromPort": f, "ToPort": t, "IpRanges": [{"CidrIp": cidr}]}
                                                for p, f, t, cidr in rules])
        if add:
            c.call("ec2", "AuthorizeSecurityGroupIngress", {"GroupId": gid, **perms(add)})
        if rm:
            c.call("ec2", "RevokeSecurityGroupIngress", {"GroupId": gid, **perms(rm)})

    def _node_groups(self, instances: list[dict]) -> set[str]:
        """The security group of each instance that carries the cluster tag (or its only one)."""
        c, out = self.aws.client, set()
        for inst in instances:
            ids = [g["groupId"] for g in _list(inst.get("groupSet"))]
            if not ids:
                continue
            if len(ids) == 1:
                out.add(ids[0])
                continue
            grps = _list(c.call("ec2", "DescribeSecurityGroups", ec2_params("GroupId", ids)).get("securityGroupInfo"))
            tagged = [g["groupId"] for g in grps if self.aws.tagging.owns(tags_of(g)) and self.aws.tagging.cluster_id]
            out.update(tagged[:1] or ids[:1])
        return out

    def _open_nodes(self, elb_gid: str, node_gids: set[str], remove_from: set[str] = frozenset()):
        """updateInstanceSecurityGroupsForLoadBalancer: node groups accept all traffic from the ELB group."""
        c = self.aws.client
        for gid in sorted(node_gids | set(remove_from)):
            grp = _list(c.call("ec2", "DescribeSecurityGroups", ec2_params("GroupId", [gid])).get("securityGroupInfo"))
            has = any(pair.get("groupId") == elb_gid for p in _list((grp[0] if grp else {}).get("ipPermissions"))
                      for pair in _list(p.get("groups")))
            perm = ec2_params("IpPermissions", [{"IpProtocol": "-1", "Groups": [{"GroupId": elb_gid}]}])
            if gid in node_gids and not has:
                c.call("ec2", "AuthorizeSecurityGroupIngress", {"GroupId": gid, **perm})
            elif gid not in node_gids and has:
                c.call("ec2", "RevokeSecurityGroupIngress", {"GroupId": gid, **perm})

    def _instances_for(self, nodes: list[dict]) -> list[dict]:
        out = []
        for n in nodes:
            pid = (n.get("spec") or {}).get("providerID", "")
            inst = None
            if pid:
                try:
                    inst = self.aws.instances_.by_id(instance_id_from_provider_id(pid))
                except ValueError:
                    inst = None
            if inst is None:
                inst = self.aws.instances_.by_name(m.name_of(n))
            out.append(inst)
        return out

    # ---- the three verbs
    def ensure(self, cluster: str, svc: dict, nodes: list[dict]) -> dict:
        spec, ann = svc.get("spec") or {}, m.annotations_of(svc)
        if spec.get("sessionAffinity", "None") != "None":
            raise ValueError(f"unsupported load balancer affinity: {spec.get('sessionAffinity')}")
        if not spec.get("ports"):
            raise ValueError("requested load balancer with no ports")
        if spec.get("loadBalancerIP"):
            raise ValueError("LoadBalancerIP cannot be specified for AWS ELB")
        if ann.get(ANN + "type", "").lower() == "nlb":
            raise ValueError("network load balancers (aws-load-balancer-type: nlb) are not supported; use a classic ELB")
        listeners = listeners_for(svc)
        internal = bool(ann.get(ANN + "internal"))
        proxy = ann.get(ANN + "proxy-protocol", "")
        if proxy and proxy != "*":
            raise ValueError(f"annotation {ANN}proxy-protocol={proxy!r} detected, but the only value supported currently is '*'")
        attrs = {"ConnectionDraining.Enabled": _s(_ann_bool(ann, "connection-draining-enabled", False)),
                 "ConnectionSettings.IdleTimeout": str(_ann_int(ann, "connection-idle-timeout", 60)),
                 "CrossZoneLoadBalancing.Enabled": _s(_ann_bool(ann, "cross-zone-load-balancing-enabled", False)),
                 "AccessLog.Enabled": _s(_ann_bool(ann, "access-log-enabled", False))}
        if ann.get(ANN + "connection-draining-timeout"):
            attrs["ConnectionDraining.Timeout"] = str(_ann_int(ann, "connection-draining-timeout", 300))
        if ann.get(ANN + "access-log-emit-interval"):
            attrs["AccessLog.EmitInterval"] = str(_ann_int(ann, "access-log-emit-interval", 60))
        for k, a in (("AccessLog.S3BucketName", "access-log-s3-bucket-name"), ("AccessLog.S3BucketPrefix", "access-log-s3-bucket-prefix")):
            if ann.get(ANN + a):
                attrs[k] = ann[ANN + a]
        instances = self._instances_for(nodes)
        subnets = self._subnets(internal)
        if not subnets:
            raise LookupError("could not find any suitable subnets for creating the ELB")
        name = lb_name(svc)
        gid = self._security_group(name, svc)
        groups = [gid] + [g.strip() for g in ann.get(ANN + "extra-security-groups", "").split(",") if g.strip()]
        ranges = spec.get("loadBalancerSourceRanges") or ["0.0.0.0/0"]
        self._set_ingress(gid, [{"IpProtocol": "tcp", "FromPort": int(p["port"]), "ToPort": int(p["port"]), "Cidrs": ranges}
                                for p in spec["ports"]] + [{"IpProtocol": "icmp", "FromPort": 3, "ToPort": 4, "Cidrs": ["0.0.0.0/0"]}])
        c = self.aws.client
        lb = self._describe(name)
        if lb is None:
            params = {"LoadBalancerName": name, **ec2_params("Listeners", listeners, "elb"),
                      **ec2_params("Subnets", subnets, "elb"), **ec2_params("SecurityGroups", groups, "elb"),
                      **ec2_params("Tags", [{"Key": k, "Value": v} for k, v in sorted(
                          self.aws.tagging.tags({TAG_SERVICE: m.key_of(svc)}).items())], "elb")}
            if internal:
                params["Scheme"] = "internal"
            c.call("elasticloadbalancing", "CreateLoadBalancer", params)
            lb = self._describe(name) or {}
        else:
            have = {(int(d["Listener"]["LoadBalancerPort"]), d["Listener"]["Protocol"].upper(), int(d["Listener"]["InstancePort"]),
                     d["Listener"].get("InstanceProtocol", "").upper(), d["Listener"].get("SSLCertificateId", ""))
                    for d in _list(lb.get("ListenerDescriptions"))}
            want = {(x["LoadBalancerPort"], x["Protocol"], x["InstancePort"], x["InstanceProtocol"], x.get("SSLCertificateId", ""))
                    for x in listeners}
            stale = sorted({h[0] for h in have - want})
            if stale:
                c.call("elasticloadbalancing", "DeleteLoadBalancerListeners",
                       {"LoadBalancerName": name, **ec2_params("LoadBalancerPorts", stale, "elb")})
            new = [x for x in listeners if (x["LoadBalancerPort"], x["Protocol"], x["InstancePort"], x["InstanceProtocol"],
                                            x.get("SSLCertificateId", "")) not in have]
            if new:
                c.call("elasticloadbalancing", "CreateLoadBalancerListeners",
                       {"LoadBalancerName": name, **ec2_params("Listeners", new, "elb")})
            cur_sub = set(_list(lb.get("Subnets")))
            if set(subnets) - cur_sub:
                c.call("elasticloadbalancing", "AttachLoadBalancerToSubnets",
                       {"LoadBalancerName": name, **ec2_params("Subnets", sorted(set(subnets) - cur_sub), "elb")})
            if cur_sub - set(subnets):
                c.call("elasticloadbalancing", "DetachLoadBalancerFromSubnets",
                       {"LoadBalancerName": name, **ec2_params("Subnets", sorted(cur_sub - set(subnets)), "elb")})
            if sorted(_list(lb.get("SecurityGroups"))) != sorted(groups):
                c.call("elasticloadbalancing", "ApplySecurityGroupsToLoadBalancer",
                       {"LoadBalancerName": name, **ec2_params("SecurityGroups", groups, "elb")})
        c.call("elasticloadbalancing", "ModifyLoadBalancerAttributes",
               {"LoadBalancerName": name, **{f"LoadBalancerAttributes.{k}": v for k, v in attrs.items()}})
        self._health_check(name, svc, listeners)
        self._register(name, lb, instances)
        self._open_nodes(gid, self._node_groups(instances))
        lb = self._describe(name) or lb
        return {"ingress": [{"hostname": lb.get("DNSName", "")}]}

    def _health_check(self, name: str, svc: dict, listeners: list[dict]):
        spec, ann = svc.get("spec") or {}, m.annotations_of(svc)
        if spec.get("externalTrafficPolicy") == "Local" and spec.get("healthCheckNodePort"):
            target = f"HTTP:{spec['healthCheckNodePort']}/healthz"
        elif listeners:
            target = f"TCP:{listeners[0]['InstancePort']}"
        else:
            return
        hc = {"HealthCheck.Target": target, "HealthCheck.HealthyThreshold": str(_ann_int(ann, "healthcheck-healthy-threshold", 2)),
              "HealthCheck.UnhealthyThreshold": str(_ann_int(ann, "healthcheck-unhealthy-threshold", 6)),
              "HealthCheck.Timeout": str(_ann_int(ann, "healthcheck-timeout", 5)),
              "HealthCheck.Interval": str(_ann_int(ann, "healthcheck-interval", 10))}
        self.aws.client.call("elasticloadbalancing", "ConfigureHealthCheck", {"LoadBalancerName": name, **hc})

    def _register(self, name: str, lb: dict, instances: list[dict]):
        c = self.aws.client
        have = {i.get("InstanceId") for i in _list((lb or {}).get("Instances"))}
        want = {i["instanceId"] for i in instances}
        if want - have:
            c.call("elasticloadbalancing", "RegisterInstancesWithLoadBalancer",
                   {"LoadBalancerName": name, **ec2_params("Instances", [{"InstanceId": i} for i in sorted(want - have)], "elb")})
        if have - want:
            c.call("elasticloadbalancing", "DeregisterInstancesFromLoadBalancer",
                   {"LoadBalancerName": name, **ec2_params("Instances", [{"InstanceId": i} for i in sorted(have - want)], "elb")})

    def update(self, cluster: str, svc: dict, nodes: list[dict]):
        name = lb_name(svc)
        lb = self._describe(name)
        if lb is None:
            raise LookupError(f"load balancer not found: {name}")
        instances = self._instances_for(nodes)
        self._register(name, lb, instances)
        groups = _list(lb.get("SecurityGroups"))
        if groups:
            self._open_nodes(groups[0], self._node_groups(instances))

    def ensure_deleted(self, cluster: str, svc: dict):
        c = self.aws.client
        name = lb_name(svc)
        lb = self._describe(name)
        if lb is None:
            return
        groups = [g for g in _list(lb.get("SecurityGroups"))]
        owned = [g for g in groups if g != self.aws.cfg.get("elbsecuritygroup")]
        if owned:
            # every group that references the ELB's group loses the rule (revoke on all node groups)
            insts = [self.aws.instances_.by_id(i.get("InstanceId")) for i in _list(lb.get("Instances"))]
            self._open_nodes(owned[0], set(), self._node_groups([i for i in insts if i]))
        c.call("elasticloadbalancing", "DeleteLoadBalancer", {"LoadBalancerName": name})
        for gid in owned:
            grp = _list(c.call("ec2", "DescribeSecurityGroups", ec2_params("GroupId", [gid])).get("securityGroupInfo"))
            if grp and self.aws.tagging.owns(tags_of(grp[0])) and grp[0].get("groupName", "").startswith("k8s-elb-"):
                deadline = time.monotonic() + 60
                while True:
                    try:
                        c.call("ec2", "DeleteSecurityGroup", {"GroupId": gid})
                        break
                    except AWSError as e:
                        if e.code != "DependencyViolation" or time.monotonic() > deadline:
                            raise
                        time.sleep(self.aws.poll)


# ----------------------------------------------------------------------------- EBS
def volume_id(kube_id: str) -> str:
    """MapToAWSVolumeID: `aws://<az>/vol-…` or `vol-…` → `vol-…`."""
    s = kube_id if kube_id.startswith("aws://") else "aws:///" + kube_id
    vid = urlsplit(s).path.strip("/")
    if not re.fullmatch(r"vol-[a-z0-9]+", vid):
        raise ValueError(f"invalid format for AWS volume ({kube_id})")
    return vid


class DeviceAllocator:
    """device_allocator.go: /dev/xvd{b,c}{a..z}, least-recently-handed-out first."""

    def __init__(self):
        self.order = {f"{a}{b}": 0 for a in "bc" for b in "abcdefghijklmnopqrstuvwxyz"}
        self.counter = 0
        self.lock = threading.Lock()

    def next(self, used: set[str]) -> str:
        for dev, _ in sorted(self.order.items(), key=lambda kv: (kv[1], kv[0])):
            if dev not in used:
                self.counter += 1
                self.order[dev] = self.counter
                return dev
        raise LookupError("no devices are available")


class Volumes:
    """EBS volumes (aws.go Create/Delete/Attach/DetachDisk)."""
    provisioner = EBS_PROVISIONER
    source_key = "awsElasticBlockStore"

    def __init__(self, aws):
        self.aws = aws
        self.allocators: dict[str, DeviceAllocator] = {}
        self.poll = 1.0

    def _describe(self, vid: str) -> dict:
        got = _list(self.aws.client.call("ec2", "DescribeVolumes", ec2_params("VolumeId", [vid])).get("volumeSet"))
        if not got:
            raise LookupError(f"volume {vid} not found")
        return got[0]

    def zones_with_instances(self) -> list[str]:
        """getCandidateZonesForDynamicVolume: zones of the running instances, masters skipped."""
        insts = self.aws.instances_.describe([{"Name": "instance-state-name", "Values": ["running"]}])
        out = set()
        for i in insts:
            t = tags_of(i)
            if "k8s.io/role/master" in t or "kubernetes.io/role/master" in t:
                continue
            if self.aws.tagging.cluster_id and not self.aws.tagging.owns(t):
                continue
            if _az(i):
                out.add(_az(i))
        return sorted(out)

    def create(self, name: str, size_gib: int, params: dict, tags: dict, pvc_name: str = "") -> str:
        zone = params.get("zone", "")
        if not zone:
            zones = [z.strip() for z in params.get("zones", "").split(",") if z.strip()] or self.zones_with_instances()
            if not zones:
                raise LookupError("no zones with instances to create the volume in")
            zone = choose_zone(zones, pvc_name or name)
        vtype = params.get("type", DEFAULT_VOLUME_TYPE).lower()
        req = {"Size": str(size_gib), "AvailabilityZone": zone, "VolumeType": vtype}
        if vtype == "io1":
            iops = int(size_gib * int(params.get("iopspergb", "0") or 0))
            req["Iops"] = str(max(100, min(iops, 20000)))
        if _truthy(params.get("encrypted", "false")):
            req["Encrypted"] = "true"
            if params.get("kmskeyid"):
                req["KmsKeyId"] = params["kmskeyid"]
        all_tags = self.aws.tagging.tags({"Name": name, **tags})
        req.update({"TagSpecification.1.ResourceType": "volume", **_tag_params(all_tags, "TagSpecification.1.Tag")})
        vol = self.aws.client.call("ec2", "CreateVolume", req)
        vid = vol["volumeId"]
        self._wait(vid, lambda v: v.get("status") == "available", "available")
        return f"aws://{zone}/{vid}"

    def delete(self, kube_id: str) -> bool:
        try:
            self.aws.client.call("ec2", "DeleteVolume", {"VolumeId": volume_id(kube_id)})
            return True
        except AWSError as e:
            if e.code == "InvalidVolume.NotFound":
                return False
            raise

    def _wait(self, vid: str, ok, what: str, timeout: float = 300):
        deadline = time.monotonic() + timeout
        while True:
            v = self._describe(vid)
            if ok(v):
                return v
            if v.get("status") == "error" or time.monotonic() > deadline:
                raise AWSError(500, "VolumeStuck", f"volume {vid} is {v.get('status')}, wanted {what}")
            time.sleep(self.poll)

    def attach(self, node: str, kube_id: str) -> str:
        vid = volume_id(kube_id)
        inst = self.aws.instances_.by_name(node)
        v = self._describe(vid)
        for a in _list(v.get("attachmentSet")):
            if a.get("instanceId") == inst["instanceId"] and a.get("status") in ("attached", "attaching"):
                self._wait(vid, lambda x: any(y.get("status") == "attached" for y in _list(x.get("attachmentSet"))), "attached")
                return a.get("device", "")
            if a.get("status") in ("attached", "attaching"):
                raise AWSError(409, "VolumeInUse", f"{vid} is attached to {a.get('instanceId')}")
        used = set()
        for bdm in _list(inst.get("blockDeviceMapping")):
            dn = bdm.get("deviceName", "")
            for pre in ("/dev/xvd", "/dev/sd"):
                if dn.startswith(pre):
                    used.add(dn[len(pre):])
        alloc = self.allocators.setdefault(node, DeviceAllocator())
        with alloc.lock:
            dev = alloc.next(used)
            self.aws.client.call("ec2", "AttachVolume", {"Device": f"/dev/xvd{dev}", "InstanceId": inst["instanceId"], "VolumeId": vid})
        v = self._wait(vid, lambda x: any(y.get("status") == "attached" for y in _list(x.get("attachmentSet"))), "attached")
        att = _list(v.get("attachmentSet"))[0]
        if att.get("device") != f"/dev/xvd{dev}" or att.get("instanceId") != inst["instanceId"]:
            raise AWSError(500, "AttachMismatch", f"disk attachment of {vid} to {node}: requested /dev/xvd{dev} on "
                           f"{inst['instanceId']}, found {att.get('device')} on {att.get('instanceId')}")
        return f"/dev/xvd{dev}"

    def detach(self, node: str, kube_id: str):
        vid = volume_id(kube_id)
        inst = self.aws.instances_.by_name(node)
        v = self._describe(vid)
        if not any(a.get("instanceId") == inst["instanceId"] for a in _list(v.get("attachmentSet"))):
            return
        self.aws.client.call("ec2", "DetachVolume", {"InstanceId": inst["instanceId"], "VolumeId": vid})
        self._wait(vid, lambda x: not _list(x.get("attachmentSet")), "detached")

    def zone(self, kube_id: str) -> str:
        return self._describe(volume_id(kube_id)).get("availabilityZone", "")

    def device_candidates(self, kube_id: str, device_path: str = "") -> list[str]:
        vid = volume_id(kube_id)
        out = [f"/dev/disk/by-id/nvme-Amazon_Elastic_Block_Store_{vid.replace('-', '')}"]
        if device_path:
            out += [device_path, device_path.replace("/dev/xvd", "/dev/sd")]
        return out

    # ---- the provisioner interface (controllers/volumes.py)
    def provision(self, name: str, gib: int, params: dict, tags: dict, pvc_name: str) -> tuple[dict, dict]:
        p = {str(k).lower(): v for k, v in params.items()}
        kid = self.create(f"kubernetes-dynamic-{name}", gib, p, tags, pvc_name)
        zone = urlsplit(kid).netloc
        return ({"volumeID": kid, "fsType": p.get("fstype", "ext4")},
                {"failure-domain.beta.kubernetes.io/zone": zone, "failure-domain.beta.kubernetes.io/region": self.aws.region})

    def delete_source(self, src: dict):
        self.delete(src["volumeID"])


def choose_zone(zones: list[str], pvc_name: str) -> str:
    """volume.ChooseZoneForVolume: a stable hash of the claim name picks the zone; StatefulSet
    claims `<claim>-<set>-<ordinal>` spread their ordinals across zones."""
    zones = sorted(zones)
    mt = re.fullmatch(r"(.*)-(\d+)", pvc_name)
    base, idx = (mt.group(1), int(mt.group(2))) if mt else (pvc_name, 0)
    h = int(hashlib.sha1(base.encode()).hexdigest()[:8], 16)
    return zones[(h + idx) % len(zones)]


# ----------------------------------------------------------------------------- provider
class AWS(Interface):
    name = PROVIDER

    def __init__(self, config=None, session=None):
        import requests
        self.cfg = parse_config(config)
        self.http = session or requests.Session()
        self.md = Metadata(self.http, self.cfg.get("metadata-url", METADATA_URL))
        self.client = Client(self.cfg, self.md, self.http)
        self.tagging = Tagging(self.cfg.get("kubernetesclusterid") or self.cfg.get("kubernetesclustertag", ""))
        self.poll = 1.0
        az = self.cfg.get("zone", "")
        if not az:
            try:
                az = self.md.get("placement/availability-zone").strip()
            except Exception as e:     # noqa: BLE001 — not on EC2 and no zone configured
                raise ValueError(f"aws: no [Global] Zone and the metadata service did not answer: {e}") from None
        if not re.fullmatch(r"[a-z]+-[a-z]+-\d+[a-z]", az):
            raise ValueError(f"aws: invalid availability zone {az!r}")
        self.zone, self.region = az, az[:-1]
        self.client.region = self.region
        self.instances_ = Instances(self)
        self._routes = Routes(self)
        self._lb = LoadBalancer(self)
        self.volumes_ = Volumes(self)
        self._vpc = self.cfg.get("vpc", "")

    def vpc_id(self) -> str:
        if not self._vpc:
            try:
                mac = self.md.get("mac").strip()
                self._vpc = self.md.get(f"network/interfaces/macs/{mac}/vpc-id").strip()
            except Exception:          # noqa: BLE001
                self._vpc = ""
        return self._vpc

    def load_balancer(self):
        return self._lb

    def instances(self):
        return self.instances_

    def routes(self):
        return self._routes if not _truthy(self.cfg.get("disableroutes", "false")) else None

    def volumes(self):
        return self.volumes_

    def zones(self):
        return Zone(self.zone, self.region)

    def has_cluster_id(self) -> bool:
        return bool(self.tagging.cluster_id)

    def zone_for_node(self, node_name: str) -> Zone:
        try:
            return Zone(_az(self.instances_.by_name(node_name)), self.region)
        except Exception:              # noqa: BLE001
            return self.zones()

    def labels_for_volume(self, pv: dict) -> dict:
        """GetLabelsForVolume: EBS volumes get their zone and the region."""
        src = (pv.get("spec") or {}).get("awsElasticBlockStore")
        if not src or src.get("volumeID", "").startswith("aws://placeholder"):
            return {}
        return {"failure-domain.beta.kubernetes.io/zone": self.volumes_.zone(src["volumeID"]),
                "failure-domain.beta.kubernetes.io/region": self.region}

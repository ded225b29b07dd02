"""A small in-memory AWS (EC2 2016-11-15 query API, classic ELB 2012-06-01, the instance
metadata service) for the provider tests: the request shapes the real services take (form POST,
Signature V4 — checked on every call), XML answers with `item`/`member` lists, EC2/ELB error
documents. Runs on its own thread (the provider's client is synchronous)."""
from __future__ import annotations

import itertools
import json
import re
import threading
import xml.sax.saxutils as su
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qsl, urlsplit

from amdkube.cloudprovider.aws import sign_v4

AK, SK = "AKIDAMDKUBETEST", "s3cr3t/amdkube+test"


def _x(tag, v, item="item"):
    if isinstance(v, dict):
        return f"<{tag}>" + "".join(_x(k, w, item) for k, w in v.items()) + f"</{tag}>"
    if isinstance(v, list):
        return f"<{tag}>" + "".join(_x(item, w, item) for w in v) + f"</{tag}>"
    if isinstance(v, bool):
        v = "true" if v else "false"
    return f"<{tag}>{su.escape(str(v))}</{tag}>"


def plist(q: dict, prefix: str, member=False) -> list:
    """`Prefix.N` scalars or `Prefix.N.Key[.…]` dicts (ELB: `Prefix.member.N…`) → list."""
    pre = prefix + (".member." if member else ".")
    rows: dict[int, object] = {}
    for k, v in q.items():
        if not k.startswith(pre):
            continue
        rest = k[len(pre):]
        idx, _, sub = rest.partition(".")
        if not idx.isdigit():
            continue
        i = int(idx)
        if not sub:
            rows[i] = v
        else:
            d = rows.setdefault(i, {})
            d[sub] = v
    return [rows[i] for i in sorted(rows)]


class EC2Error(Exception):
    def __init__(self, code, msg, status=400):
        super().__init__(msg)
        self.code, self.msg, self.status = code, msg, status


class FakeAWS:
    def __init__(self, region="us-east-1", cluster="mi355x"):
        self.region, self.cluster = region, cluster
        self.lock = threading.RLock()
        self.ids = itertools.count(1)
        self.instances: dict[str, dict] = {}
        self.subnets: dict[str, dict] = {}
        self.groups: dict[str, dict] = {}
        self.tables: dict[str, dict] = {}
        self.volumes: dict[str, dict] = {}
        self.lbs: dict[str, dict] = {}
        self.calls: list[str] = []
        self.bad_signatures = 0
        self.self_id = None
        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), self._handler())
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}"

    def _id(self, pre):
        return f"{pre}-{next(self.ids):08x}"

    def ctag(self):
        return {"key": f"kubernetes.io/cluster/{self.cluster}", "value": "owned"}

    # ------------------------------------------------------------------ fixtures
    def add_instance(self, ip, az="us-east-1a", itype="p5.48xlarge", public=None, groups=None, state="running"):
        iid = self._id("i")
        dns = f"ip-{ip.replace('.', '-')}.ec2.internal"
        inst = {"instanceId": iid, "instanceType": itype, "privateDnsName": dns, "privateIpAddress": ip,
                "placement": {"availabilityZone": az}, "instanceState": {"code": "16", "name": state},
                "networkInterfaceSet": [{"status": "in-use", "privateIpAddressesSet": [{"privateIpAddress": ip}]}],
                "groupSet": [{"groupId": g} for g in (groups or [])], "blockDeviceMapping": [{"deviceName": "/dev/xvda"}],
                "tagSet": [self.ctag()], "sourceDestCheck": True}
        if public:
            inst["ipAddress"], inst["dnsName"] = public, f"ec2-{public.replace('.', '-')}.compute-1.amazonaws.com"
        self.instances[iid] = inst
        if self.self_id is None:
            self.self_id = iid
        return inst

    def add_subnet(self, az, role=None, tagged=True):
        sid = self._id("subnet")
        tags = [self.ctag()] if tagged else []
        if role:
            tags.append({"key": role, "value": "1"})
        self.subnets[sid] = {"subnetId": sid, "vpcId": "vpc-1", "availabilityZone": az, "tagSet": tags}
        return sid

    def add_group(self, name, tagged=True):
        gid = self._id("sg")
        self.groups[gid] = {"groupId": gid, "groupName": name, "vpcId": "vpc-1", "ipPermissions": [],
                            "tagSet": [self.ctag()] if tagged else []}
        return gid

    def add_route_table(self, tagged=True):
        rid = self._id("rtb")
        self.tables[rid] = {"routeTableId": rid, "vpcId": "vpc-1", "routeSet": [], "tagSet": [self.ctag()] if tagged else []}
        return rid

    def start(self):
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()
        return self

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()

    def config(self, **extra):
        return {"Global": {"Zone": "us-east-1a", "KubernetesClusterID": self.cluster, "VPC": "vpc-1",
                           "ec2-endpoint": self.url + "/ec2/", "elb-endpoint": self.url + "/elb/",
                           "metadata-url": self.url + "/latest/meta-data/", **extra}}

    # ------------------------------------------------------------------ HTTP
    def _handler(self):
        aws = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, text, ctype="text/xml"):
                data = text.encode()
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def do_GET(self):
                u = urlsplit(self.path)
                if not u.path.startswith("/latest/meta-data/"):
                    return self._send(404, "not found", "text/plain")
                code, text = aws.metadata(u.path[len("/latest/meta-data/"):])
                self._send(code, text, "text/plain")

            def do_POST(self):
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n)
                svc = "ec2" if self.path.startswith("/ec2") else "elasticloadbalancing"
                auth = self.headers.get("Authorization", "")
                mt = re.match(r"AWS4-HMAC-SHA256 Credential=([^/]+)/(\d{8})/([^/]+)/([^/]+)/aws4_request, SignedHeaders=([^,]+), Signature=(\w+)", auth)
                ok = False
                if mt and mt.group(1) == AK and mt.group(3) == aws.region and mt.group(4) == svc:
                    hdrs = {h: self.headers.get(h, "") for h in mt.group(5).split(";") if h not in ("host", "x-amz-date", "x-amz-security-token")}
                    want = sign_v4("POST", f"http://{self.headers.get('Host')}{self.path}", {"Host": self.headers.get("Host"), **hdrs},
                                   body, aws.region, svc, AK, SK, self.headers.get("X-Amz-Date", ""),
                                   self.headers.get("X-Amz-Security-Token", ""))
                    ok = want["Authorization"] == auth
                q = dict(parse_qsl(body.decode(), keep_blank_values=True))
                act = q.get("Action", "")
                elb = svc != "ec2"
                if not ok:
                    aws.bad_signatures += 1
                    return self._send(403, aws.error_doc("SignatureDoesNotMatch", "bad signature", elb))
                with aws.lock:
                    aws.calls.append(act)
                    try:
                        fn = getattr(aws, ("elb_" if elb else "ec2_") + act)
                        out = fn(q)
                    except EC2Error as e:
                        return self._send(e.status, aws.error_doc(e.code, e.msg, elb))
                    except AttributeError:
                        return self._send(400, aws.error_doc("InvalidAction", act, elb))
                if elb:
                    doc = f'<{act}Response xmlns="http://elasticloadbalancing.amazonaws.com/doc/2012-06-01/">' + \
                          _x(f"{act}Result", out or {}, "member") + "<ResponseMetadata><RequestId>r</RequestId></ResponseMetadata>" + \
                          f"</{act}Response>"
                else:
                    inner = "".join(_x(k, v) for k, v in (out or {}).items())
                    doc = f'<{act}Response xmlns="http://ec2.amazonaws.com/doc/2016-11-15/"><requestId>r</requestId>{inner}</{act}Response>'
                self._send(200, doc)
        return H

    @staticmethod
    def error_doc(code, msg, elb):
        if elb:
            return f"<ErrorResponse><Error><Type>Sender</Type><Code>{code}</Code><Message>{su.escape(msg)}</Message></Error></ErrorResponse>"
        return f"<Response><Errors><Error><Code>{code}</Code><Message>{su.escape(msg)}</Message></Error></Errors><RequestID>r</RequestID></Response>"

    def metadata(self, path):
        inst = self.instances.get(self.self_id) or {}
        table = {"placement/availability-zone": inst.get("placement", {}).get("availabilityZone", ""),
                 "instance-id": inst.get("instanceId", ""), "local-hostname": inst.get("privateDnsName", ""),
                 "mac": "0a:00:00:00:00:01", "network/interfaces/macs/0a:00:00:00:00:01/vpc-id": "vpc-1",
                 "iam/security-credentials/": "gpu-node-role",
                 "iam/security-credentials/gpu-node-role": json.dumps({"AccessKeyId": AK, "SecretAccessKey": SK, "Token": "tok-1",
                                                                       "Expiration": "2099-01-01T00:00:00Z"})}
        return (200, table[path]) if path in table else (404, "")

    # ------------------------------------------------------------------ EC2
    def _filters(self, q):
        return {f["Name"]: [v for k, v in sorted(f.items()) if k.startswith("Value.")] for f in plist(q, "Filter")}

    @staticmethod
    def _match(obj, flt, fields):
        for name, vals in flt.items():
            if name == "tag-key":
                if not any(t["key"] in vals for t in obj.get("tagSet") or []):
                    return False
                continue
            if fields(name) not in vals:
                return False
        return True

    def ec2_DescribeInstances(self, q):
        ids = plist(q, "InstanceId")
        for i in ids:
            if i not in self.instances:
                raise EC2Error("InvalidInstanceID.NotFound", f"The instance ID '{i}' does not exist")
        flt = self._filters(q)
        keys = {"private-dns-name": "privateDnsName", "instance-id": "instanceId"}
        got = [i for i in self.instances.values() if (not ids or i["instanceId"] in ids) and self._match(
            i, flt, lambda n, i=i: i["instanceState"]["name"] if n == "instance-state-name" else i.get(keys.get(n, n)))]
        return {"reservationSet": [{"reservationId": f"r-{i['instanceId']}", "instancesSet": [i]} for i in got]}

    def ec2_ModifyInstanceAttribute(self, q):
        self.instances[q["InstanceId"]]["sourceDestCheck"] = q.get("SourceDestCheck.Value") == "true"
        return {"return": "true"}

    def ec2_DescribeRouteTables(self, q):
        flt = self._filters(q)
        return {"routeTableSet": [t for t in self.tables.values()
                                  if self._match(t, flt, lambda n, t=t: t["routeTableId"] if n == "route-table-id" else t.get(n))]}

    def ec2_CreateRoute(self, q):
        t = self.tables[q["RouteTableId"]]
        if any(r["destinationCidrBlock"] == q["DestinationCidrBlock"] for r in t["routeSet"]):
            raise EC2Error("RouteAlreadyExists", "route exists")
        t["routeSet"].append({"destinationCidrBlock": q["DestinationCidrBlock"], "instanceId": q["InstanceId"], "state": "active"})
        return {"return": "true"}

    def ec2_DeleteRoute(self, q):
        t = self.tables[q["RouteTableId"]]
        before = len(t["routeSet"])
        t["routeSet"] = [r for r in t["routeSet"] if r["destinationCidrBlock"] != q["DestinationCidrBlock"]]
        if len(t["routeSet"]) == before:
            raise EC2Error("InvalidRoute.NotFound", "no route")
        return {"return": "true"}

    def ec2_DescribeSubnets(self, q):
        flt = self._filters(q)
        return {"subnetSet": [s for s in self.subnets.values()
                              if self._match(s, flt, lambda n, s=s: s["vpcId"] if n == "vpc-id" else s.get(n))]}

    def ec2_DescribeSecurityGroups(self, q):
        ids, flt = plist(q, "GroupId"), self._filters(q)
        keys = {"group-name": "groupName", "vpc-id": "vpcId"}
        return {"securityGroupInfo": [g for g in self.groups.values() if (not ids or g["groupId"] in ids)
                                      and self._match(g, flt, lambda n, g=g: g.get(keys.get(n, n)))]}

    def ec2_CreateSecurityGroup(self, q):
        if any(g["groupName"] == q["GroupName"] for g in self.groups.values()):
            raise EC2Error("InvalidGroup.Duplicate", "exists")
        gid = self.add_group(q["GroupName"], tagged=False)
        self.groups[gid]["groupDescription"] = q.get("GroupDescription", "")
        return {"groupId": gid}

    def ec2_CreateTags(self, q):
        for rid in plist(q, "ResourceId"):
            obj = self.groups.get(rid) or self.volumes.get(rid) or self.instances.get(rid)
            for t in plist(q, "Tag"):
                obj.setdefault("tagSet", []).append({"key": t["Key"], "value": t.get("Value", "")})
        return {"return": "true"}

    def _perms(self, q):
        out = []
        for p in plist(q, "IpPermissions"):
            proto = p["IpProtocol"]
            fr, to = int(p.get("FromPort", 0)), int(p.get("ToPort", 0))
            cidrs = [v for k, v in sorted(p.items()) if re.fullmatch(r"IpRanges\.\d+\.CidrIp", k)]
            grps = [v for k, v in sorted(p.items()) if re.fullmatch(r"Groups\.\d+\.GroupId", k)]
            out.append((proto, fr, to, cidrs, grps))
        return out

    def ec2_AuthorizeSecurityGroupIngress(self, q):
        g = self.groups[q["GroupId"]]
        for proto, fr, to, cidrs, grps in self._perms(q):
            g["ipPermissions"].append({"ipProtocol": proto, "fromPort": fr, "toPort": to,
                                       "ipRanges": [{"cidrIp": c} for c in cidrs], "groups": [{"groupId": x} for x in grps]})
        return {"return": "true"}

    def ec2_RevokeSecurityGroupIngress(self, q):
        g = self.groups[q["GroupId"]]
        for proto, fr, to, cidrs, grps in self._perms(q):
            keep = []
            for p in g["ipPermissions"]:
                if p["ipProtocol"] == proto and (proto == "-1" or (p["fromPort"], p["toPort"]) == (fr, to)):
                    p = dict(p, ipRanges=[r for r in p["ipRanges"] if r["cidrIp"] not in cidrs],
                             groups=[x for x in p["groups"] if x["groupId"] not in grps])
                    if not p["ipRanges"] and not p["groups"]:
                        continue
                keep.append(p)
            g["ipPermissions"] = keep
        return {"return": "true"}

    def ec2_DeleteSecurityGroup(self, q):
        gid = q["GroupId"]
        if any(gid in [x["groupId"] for x in lb["SecurityGroups_"]] for lb in self.lbs.values()):
            raise EC2Error("DependencyViolation", "in use by a load balancer")
        self.groups.pop(gid, None)
        return {"return": "true"}

    def ec2_CreateVolume(self, q):
        vid = self._id("vol")
        tags = [{"key": t["Key"], "value": t.get("Value", "")} for t in plist(q, "TagSpecification.1.Tag")]
        v = {"volumeId": vid, "size": q["Size"], "availabilityZone": q["AvailabilityZone"], "status": "available",
             "volumeType": q.get("VolumeType", "standard"), "iops": q.get("Iops", ""), "encrypted": q.get("Encrypted", "false"),
             "attachmentSet": [], "tagSet": tags}
        self.volumes[vid] = v
        return {k: v[k] for k in ("volumeId", "size", "availabilityZone", "status", "volumeType")}

    def ec2_DescribeVolumes(self, q):
        ids = plist(q, "VolumeId")
        for i in ids:
            if i not in self.volumes:
                raise EC2Error("InvalidVolume.NotFound", f"The volume '{i}' does not exist.")
        return {"volumeSet": [v for v in self.volumes.values() if not ids or v["volumeId"] in ids]}

    def ec2_AttachVolume(self, q):
        v, inst = self.volumes[q["VolumeId"]], self.instances[q["InstanceId"]]
        if v["attachmentSet"]:
            raise EC2Error("VolumeInUse", "attached")
        if v["availabilityZone"] != inst["placement"]["availabilityZone"]:
            raise EC2Error("InvalidVolume.ZoneMismatch", "zone mismatch")
        v["attachmentSet"] = [{"volumeId": v["volumeId"], "instanceId": inst["instanceId"], "device": q["Device"], "status": "attached"}]
        v["status"] = "in-use"
        inst["blockDeviceMapping"].append({"deviceName": q["Device"], "ebs": {"volumeId": v["volumeId"]}})
        return {"volumeId": v["volumeId"], "instanceId": inst["instanceId"], "device": q["Device"], "status": "attaching"}

    def ec2_DetachVolume(self, q):
        v, inst = self.volumes[q["VolumeId"]], self.instances[q["InstanceId"]]
        v["attachmentSet"], v["status"] = [], "available"
        inst["blockDeviceMapping"] = [b for b in inst["blockDeviceMapping"] if (b.get("ebs") or {}).get("volumeId") != v["volumeId"]]
        return {"volumeId": v["volumeId"], "status": "detaching"}

    def ec2_DeleteVolume(self, q):
        v = self.volumes.get(q["VolumeId"])
        if v is None:
            raise EC2Error("InvalidVolume.NotFound", "no such volume")
        if v["attachmentSet"]:
            raise EC2Error("VolumeInUse", "attached")
        del self.volumes[q["VolumeId"]]
        return {"return": "true"}

    # ------------------------------------------------------------------ ELB
    def _lb(self, name):
        lb = self.lbs.get(name)
        if lb is None:
            raise EC2Error("LoadBalancerNotFound", f"There is no ACTIVE Load Balancer named '{name}'")
        return lb

    @staticmethod
    def _listener(d):
        return {k: d[k] for k in ("Protocol", "LoadBalancerPort", "InstanceProtocol", "InstancePort", "SSLCertificateId") if k in d}

    def elb_DescribeLoadBalancers(self, q):
        names = plist(q, "LoadBalancerNames", True)
        out = []
        for n in names or list(self.lbs):
            lb = self._lb(n)
            out.append({"LoadBalancerName": n, "DNSName": lb["DNSName"], "Scheme": lb["Scheme"],
                        "ListenerDescriptions": [{"Listener": li, "PolicyNames": []} for li in lb["Listeners"]],
                        "Subnets": lb["Subnets"], "SecurityGroups": [x["groupId"] for x in lb["SecurityGroups_"]],
                        "Instances": [{"InstanceId": i} for i in lb["Instances"]], "HealthCheck": lb.get("HealthCheck", {})})
        return {"LoadBalancerDescriptions": out}

    def elb_CreateLoadBalancer(self, q):
        n = q["LoadBalancerName"]
        if n in self.lbs:
            raise EC2Error("DuplicateLoadBalancerName", n)
        scheme = q.get("Scheme", "internet-facing")
        self.lbs[n] = {"DNSName": f"{'internal-' if scheme == 'internal' else ''}{n}-1234.{self.region}.elb.amazonaws.com",
                       "Scheme": scheme, "Listeners": [self._listener(d) for d in plist(q, "Listeners", True)],
                       "Subnets": plist(q, "Subnets", True), "SecurityGroups_": [{"groupId": g} for g in plist(q, "SecurityGroups", True)],
                       "Instances": [], "Tags": {t["Key"]: t.get("Value", "") for t in plist(q, "Tags", True)}, "Attributes": {}}
        return {"DNSName": self.lbs[n]["DNSName"]}

    def elb_DeleteLoadBalancer(self, q):
        self.lbs.pop(q["LoadBalancerName"], None)
        return {}

    def elb_CreateLoadBalancerListeners(self, q):
        lb = self._lb(q["LoadBalancerName"])
        lb["Listeners"] += [self._listener(d) for d in plist(q, "Listeners", True)]
        return {}

    def elb_DeleteLoadBalancerListeners(self, q):
        lb = self._lb(q["LoadBalancerName"])
        ports = set(plist(q, "LoadBalancerPorts", True))
        lb["Listeners"] = [li for li in lb["Listeners"] if str(li["LoadBalancerPort"]) not in ports]
        return {}

    def elb_AttachLoadBalancerToSubnets(self, q):
        lb = self._lb(q["LoadBalancerName"])
        lb["Subnets"] = sorted(set(lb["Subnets"]) | set(plist(q, "Subnets", True)))
        return {"Subnets": lb["Subnets"]}

    def elb_DetachLoadBalancerFromSubnets(self, q):
        lb = self._lb(q["LoadBalancerName"])
        lb["Subnets"] = sorted(set(lb["Subnets"]) - set(plist(q, "Subnets", True)))
        return {"Subnets": lb["Subnets"]}

    def elb_ApplySecurityGroupsToLoadBalancer(self, q):
        lb = self._lb(q["LoadBalancerName"])
        lb["SecurityGroups_"] = [{"groupId": g} for g in plist(q, "SecurityGroups", True)]
        return {"SecurityGroups": [x["groupId"] for x in lb["SecurityGroups_"]]}

    def elb_RegisterInstancesWithLoadBalancer(self, q):
        lb = self._lb(q["LoadBalancerName"])
        for d in plist(q, "Instances", True):
            if d["InstanceId"] not in lb["Instances"]:
                lb["Instances"].append(d["InstanceId"])
        return {"Instances": [{"InstanceId": i} for i in lb["Instances"]]}

    def elb_DeregisterInstancesFromLoadBalancer(self, q):
        lb = self._lb(q["LoadBalancerName"])
        drop = {d["InstanceId"] for d in plist(q, "Instances", True)}
        lb["Instances"] = [i for i in lb["Instances"] if i not in drop]
        return {"Instances": [{"InstanceId": i} for i in lb["Instances"]]}

    def elb_ConfigureHealthCheck(self, q):
        lb = self._lb(q["LoadBalancerName"])
        lb["HealthCheck"] = {k.split(".", 1)[1]: v for k, v in q.items() if k.startswith("HealthCheck.")}
        return {"HealthCheck": lb["HealthCheck"]}

    def elb_ModifyLoadBalancerAttributes(self, q):
        lb = self._lb(q["LoadBalancerName"])
        lb["Attributes"].update({k.split(".", 1)[1]: v for k, v in q.items() if k.startswith("LoadBalancerAttributes.")})
        return {"LoadBalancerName": q["LoadBalancerName"]}

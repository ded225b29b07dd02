"""Advanced auditing (reference staging/src/k8s.io/apiserver/pkg/audit/policy/checker_test.go
rule matching; plugin/pkg/audit/log backend output; request.go event contents)."""
import json

from amdkube.apiserver.audit import level_for
from amdkube.localcluster import LocalCluster

POLICY = """
apiVersion: audit.k8s.io/v1beta1
kind: Policy
omitStages: ["RequestReceived"]
rules:
- level: None
  users: ["system:kube-proxy"]
- level: None
  resources: [{group: "", resources: ["events"]}]
- level: RequestResponse
  resources: [{group: "", resources: ["pods", "pods/status"]}]
  namespaces: ["gpu"]
- level: Request
  verbs: ["create", "update", "patch", "delete"]
- level: Metadata
"""


def test_policy_rule_matching(tmp_path):
    import yaml
    pol = yaml.safe_load(POLICY)
    u = {"name": "alice", "groups": ["system:authenticated"]}
    assert level_for(pol, {"name": "system:kube-proxy"}, "get", "", "pods", "", "gpu", "x", "")[0] == "None"
    assert level_for(pol, u, "list", "", "events", "", "default", "", "")[0] == "None"
    assert level_for(pol, u, "get", "", "pods", "status", "gpu", "x", "")[0] == "RequestResponse"
    assert level_for(pol, u, "get", "", "pods", "", "default", "x", "")[0] == "Metadata"
    assert level_for(pol, u, "create", "apps", "deployments", "", "default", "", "")[0] == "Request"
    lvl, omit = level_for(pol, u, "get", "", "nodes", "", "", "n", "")
    assert lvl == "Metadata" and omit == {"RequestReceived"}


async def test_audit_log_records_requests(tmp_path):
    pol = tmp_path / "policy.yaml"
    pol.write_text(POLICY)
    log = tmp_path / "audit.log"
    async with LocalCluster(gpus="none", with_kubelet=False, with_controllers=False,
                            api_kw={"audit_log_path": str(log), "audit_policy_file": str(pol)}) as lc:
        c = lc.client
        await c.create({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "gpu"}})
        await c.create({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p"},
                        "spec": {"containers": [{"name": "c", "image": "busybox"}]}}, "gpu")
        await c.get("pods", "p", "gpu")
        await c.delete("pods", "p", "gpu", grace=0)
    events = [json.loads(line) for line in log.read_text().splitlines()]
    assert all(e["stage"] != "RequestReceived" for e in events)      # omitStages
    pod_get = [e for e in events if e["verb"] == "get" and e.get("objectRef", {}).get("resource") == "pods"]
    assert pod_get and pod_get[0]["level"] == "RequestResponse" and pod_get[0]["responseObject"]["metadata"]["name"] == "p"
    assert pod_get[0]["responseStatus"]["code"] == 200 and pod_get[0]["user"]["username"] == "system:apiserver"
    ns_create = [e for e in events if e["verb"] == "create" and e["objectRef"]["resource"] == "namespaces"][0]
    assert ns_create["level"] == "Request" and ns_create["requestObject"]["metadata"]["name"] == "gpu"
    assert "responseObject" not in ns_create and ns_create["auditID"]

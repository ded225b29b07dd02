"""Reference documentation generators: the reference's cmd/gendocs (kubectl markdown),
cmd/genkubedocs (per-component markdown), cmd/genman (man pages) and cmd/genyaml (kubectl
YAML), over this build's argparse parsers and the kubectl help table (kubectl/help.py).

  python -m amdkube gendocs  [--out DIR] [--what kubectl|components|all]   # markdown
  python -m amdkube genman   [--out DIR]                                    # roff man(1)
  python -m amdkube genyaml  [--out DIR]                                    # kubectl YAML

The component parsers are built inside each component's entry function; capture_parser()
runs the entry with parse_args intercepted, so nothing starts and no flag needs repeating.
"""
from __future__ import annotations

import argparse
import datetime
import os
import sys

import yaml


class _Captured(Exception):
    def __init__(self, parser):
        super().__init__("captured")
        self.parser = parser


def capture_parser(entry) -> argparse.ArgumentParser | None:
    """The first ArgumentParser `entry([])` parses with (nothing runs past parsing)."""
    saved = argparse.ArgumentParser.parse_args, argparse.ArgumentParser.parse_known_args

    def grab(self, *a, **kw):
        raise _Captured(self)
    argparse.ArgumentParser.parse_args = grab
    argparse.ArgumentParser.parse_known_args = grab
    try:
        entry([])
    except _Captured as c:
        return c.parser
    except SystemExit:
        return None
    finally:
        argparse.ArgumentParser.parse_args, argparse.ArgumentParser.parse_known_args = saved
    return None


def _options(parser: argparse.ArgumentParser, skip: set[str] = frozenset()) -> list[dict]:
    out = []
    for act in parser._actions:
        if not act.option_strings or isinstance(act, argparse._HelpAction):
            continue
        longs = [o for o in act.option_strings if o.startswith("--")]
        shorts = [o for o in act.option_strings if not o.startswith("--")]
        name = (longs or shorts)[0].lstrip("-")
        if name in skip:
            continue
        d = {"name": name}
        if longs and shorts:
            d["shorthand"] = shorts[0].lstrip("-")
        dv = act.default
        if dv not in (None, argparse.SUPPRESS, False, [], "") and not callable(dv):
            d["default_value"] = str(dv)
        if act.help and act.help != argparse.SUPPRESS:
            d["usage"] = act.help.replace("%%", "%")
        out.append(d)
    return out


def kubectl_docs() -> list[dict]:
    """One doc per kubectl command (genyaml's cmdDoc shape), the root first."""
    from ..kubectl import help as kh
    from ..kubectl.main import parser
    root = parser()
    sub = next(a for a in root._actions if isinstance(a, argparse._SubParsersAction))
    inherited = _options(root)
    global_names = {o["name"] for o in inherited}
    docs = [{"name": "kubectl", "synopsis": "kubectl controls the amdkube cluster manager",
             "description": kh.overview(), "options": inherited,
             "see_also": [f"kubectl {c}" for c in sorted(sub.choices)]}]
    for name in sorted(sub.choices):
        sp = sub.choices[name]
        d = {"name": f"kubectl {name}", "synopsis": kh.short(name), "description": kh.long_desc(name),
             "options": _options(sp, global_names), "inherited_options": inherited}
        if kh.examples(name).strip():
            d["example"] = kh.examples(name)
        d["see_also"] = ["kubectl"]
        docs.append(d)
    return docs


COMPONENT_SYNOPSIS = {
    "kube-apiserver": "Serves the REST and watch API over the embedded MVCC store, with authentication, "
                      "authorization, admission (ResourceV2 turns amd.com/gpu limits into device-granular "
                      "requests) and the aggregator.",
    "kube-scheduler": "Places pods on nodes; for extended resources it chooses the exact GPU devices "
                      "(xGMI/NUMA topology scoring, reserve-on-assume) and binds them with the node.",
    "kube-controller-manager": "Runs the controllers (replication, deployments, daemonsets, jobs, node "
                               "lifecycle, garbage collection, volumes, certificates, ...).",
    "kubelet": "The node agent: admits pods through the device manager (AdmitPod), starts their containers "
               "on the CRI runtime with the GPU devices the plugins return (InitContainer), and reports node "
               "status including every GPU's health and attributes.",
    "kube-proxy": "Programs service load balancing (iptables, ipvs or userspace) on the node.",
    "kube-dns": "Cluster DNS for services and pods.",
    "kubeadm": "Bootstraps a cluster: init (as phases), join, token, config, upgrade, reset.",
    "amd-device-plugin": "Advertises the node's MI355X GPUs (or their partitions) over the device-plugin "
                         "v1alpha2 API with health from amd-smi, and tells the kubelet which device nodes and "
                         "environment a container needs.",
    "amdgpu-exporter": "Prometheus exporter of amd-smi GPU metrics attributed to pods.",
    "cloud-controller-manager": "Cloud-specific controllers (node initialisation, routes, load balancers, "
                                "PV labels) behind --cloud-provider.",
    "hollow-node": "A kubemark hollow node: a real kubelet and AMD device plugin over a simulated 8xMI355X.",
    "local-up": "Starts a single-node cluster on this host (local-up-cluster).",
    "metrics-server": "Serves metrics.k8s.io node and pod metrics from kubelet summaries.",
    "gke-certificates-controller": "Signs approved certificate signing requests through an external signing webhook.",
    "rktshim": "CRI runtime that runs pods as rkt pods through the rkt command line.",
    "rocshim": "The CRI runtime: pause sandboxes and process containers with only their GPUs' device nodes.",
    "cluster-proportional-autoscaler": "Scales a workload (kube-dns) linearly or by ladder steps with the cluster's "
                                       "nodes, cores and GPUs.",
    "ip-masq-agent": "Keeps the nat IP-MASQ-AGENT chain: pod traffic to non-masquerade CIDRs keeps its source, the rest "
                     "is masqueraded.",
    "dashboard": "Web UI over the cluster: nodes with their MI355X GPUs, workloads, pods with logs, services, events.",
    "log-store": "The elasticsearch-logging service: an Elasticsearch-compatible bulk/search API over per-day log indices.",
    "log-shipper": "Tails container and component logs on the node, adds pod metadata and ships them to the log store.",
}


def component_docs() -> list[dict]:
    from .components import COMPONENTS
    seen, docs = {}, []
    for name in sorted(COMPONENTS, key=lambda n: (not n.startswith("kube"), n)):   # kube-* names win over aliases
        fn = COMPONENTS[name]
        if fn in seen or name in GENERATORS:
            continue
        seen[fn] = name
        p = capture_parser(fn)
        if p is None:
            continue
        aliases = sorted(n for n, f in COMPONENTS.items() if f is fn and n != name)
        syn = COMPONENT_SYNOPSIS.get(name) or (p.description or f"amdkube {name}").splitlines()[0]
        docs.append({"name": name, "synopsis": syn.split(": ")[0].split(". ")[0],
                     "description": p.description or syn, "options": _options(p),
                     "see_also": [f"amdkube {a}" for a in aliases]})
    return docs


def _fname(name: str, ext: str) -> str:
    return name.replace(" ", "_") + ext


def render_markdown(d: dict) -> str:
    out = [f"## {d['name']}", "", d.get("synopsis", ""), "", "### Synopsis", "", d.get("description", "").strip(), ""]
    if d.get("example"):
        out += ["### Examples", "", "```", d["example"], "```", ""]
    for key, title in (("options", "Options"), ("inherited_options", "Options inherited from parent commands")):
        if d.get(key):
            out += [f"### {title}", "", "```"]
            for o in d[key]:
                flag = (f"-{o['shorthand']}, " if o.get("shorthand") else "    ") + f"--{o['name']}"
                if o.get("default_value") is not None:
                    flag += f"={o['default_value']}"
                out.append(f"  {flag:<44} {o.get('usage', '')}".rstrip())
            out += ["```", ""]
    if d.get("see_also"):
        out += ["### SEE ALSO", ""] + [f"* [{s}]({_fname(s, '.md')})" for s in d["see_also"]] + [""]
    return "\n".join(out)


def _roff(s: str) -> str:
    return s.replace("\\", "\\\\").replace("-", "\\-").replace("\n.", "\n\\&.")


def render_man(d: dict, section: int = 1) -> str:
    title = d["name"].replace(" ", "-").upper()
    date = datetime.date.today().strftime("%b %Y")
    out = [f'.TH "{title}" "{section}" "{date}" "amdkube" "amdkube Manuals"', ".nh", ".ad l", "",
           ".SH NAME", _roff(f"{d['name'].replace(' ', '-')} - {d.get('synopsis', '')}"), "",
           ".SH SYNOPSIS", f".B {_roff(d['name'])}", "[OPTIONS]", "", ".SH DESCRIPTION", _roff(d.get("description", "")), ""]
    for key, title_ in (("options", "OPTIONS"), ("inherited_options", "OPTIONS INHERITED FROM PARENT COMMANDS")):
        if d.get(key):
            out.append(f".SH {title_}")
            for o in d[key]:
                flag = (f"\\fB\\-{o['shorthand']}\\fP, " if o.get("shorthand") else "") + f"\\fB\\-\\-{_roff(o['name'])}\\fP"
                if o.get("default_value") is not None:
                    flag += f"={_roff(o['default_value'])}"
                out += [".PP", flag, ".RS", _roff(o.get("usage", "")) or ".", ".RE", ""]
    if d.get("example"):
        out += [".SH EXAMPLE", ".PP", ".RS", ".nf", _roff(d["example"]), ".fi", ".RE", ""]
    if d.get("see_also"):
        out += [".SH SEE ALSO", ", ".join(f"\\fB{_roff(s.replace(' ', '-'))}(1)\\fP" for s in d["see_also"]), ""]
    return "\n".join(out)


def write(docs: list[dict], out_dir: str, fmt: str) -> list[str]:
    os.makedirs(out_dir, exist_ok=True)
    written = []
    for d in docs:
        if fmt == "md":
            path, text = os.path.join(out_dir, _fname(d["name"], ".md")), render_markdown(d)
        elif fmt == "man":
            path, text = os.path.join(out_dir, d["name"].replace(" ", "-") + ".1"), render_man(d)
        elif fmt == "yaml":
            path = os.path.join(out_dir, _fname(d["name"], ".yaml"))
            text = yaml.safe_dump(d, sort_keys=False, default_flow_style=False)
        else:
            raise ValueError(f"unknown format {fmt!r}")
        with open(path, "w") as f:
            f.write(text)
        written.append(path)
    return written


def _main(argv, fmt: str, default_out: str):
    ap = argparse.ArgumentParser(f"amdkube gen{fmt}", description="Generate reference documentation.")
    ap.add_argument("--out", default=default_out, help="output directory")
    ap.add_argument("--what", default="all", choices=("kubectl", "components", "all"), help="which commands to document")
    a = ap.parse_args(argv)
    docs = []
    if a.what in ("kubectl", "all"):
        docs += kubectl_docs()
    if a.what in ("components", "all"):
        docs += component_docs()
    paths = write(docs, a.out, fmt)
    print(f"wrote {len(paths)} {fmt} files to {a.out}", file=sys.stderr)
    return 0


def gendocs(argv):
    return _main(argv, "md", "docs/generated/md")


def genman(argv):
    return _main(argv, "man", "docs/generated/man/man1")


def genyaml(argv):
    return _main(argv, "yaml", "docs/generated/yaml")


GENERATORS = {"gendocs": gendocs, "genkubedocs": gendocs, "genman": genman, "genyaml": genyaml}

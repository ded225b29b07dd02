"""Command help for kubectl: one short line, a long description and indented examples per
command (the reference keeps them on each cobra command, pkg/kubectl/cmd/*.go, normalised by
pkg/kubectl/cmd/templates and checked by cmd/clicheck → pkg/kubectl/cmd/util/sanity/
cmd_sanity.go). `kubectl help [command]`, `kubectl <command> --help` and
`python -m amdkube gendocs` all read this table; tests/test_clicheck.py applies the
reference's conventions to it (trimmed long text, examples indented two spaces with `#`
comments, lowercase-dash flag names)."""
from __future__ import annotations

import textwrap

INDENT = "  "

# command → (short, long, examples)
HELP: dict[str, tuple[str, str, str]] = {
    "get": ("Display one or many resources",
            "Prints a table of the most important fields of the named resources, or of every resource of a type. "
            "GPU columns (requested and assigned amd.com/gpu devices, node GPU health) are part of the default "
            "pod and node tables. Use -o json|yaml|name|wide|jsonpath=... for other formats and -w to keep "
            "watching.",
            "# List all pods in the current namespace, with their GPU assignment\n"
            "kubectl get pods\n"
            "# List nodes with their healthy/total MI355X counts\n"
            "kubectl get nodes\n"
            "# One pod as YAML\n"
            "kubectl get pod trainer -o yaml\n"
            "# Pods on every namespace that carry a label\n"
            "kubectl get pods -A -l app=train"),
    "describe": ("Show details of a specific resource or group of resources",
                 "Prints a detailed description of the selected resources, including related events. For pods "
                 "this lists each extended-resource request with its assigned GPU IDs; for nodes the per-device "
                 "health and attributes (type, HBM size, NUMA node, xGMI hive).",
                 "# Describe a node and its GPUs\n"
                 "kubectl describe node mi355x-0\n"
                 "# Describe every pod with a label\n"
                 "kubectl describe pods -l app=train"),
    "create": ("Create a resource from a file or from stdin",
               "Creates the objects in the given JSON or YAML files (or stdin with -f -). Subcommands generate "
               "common objects directly: namespace, configmap, secret, serviceaccount, deployment, job, "
               "priorityclass, quota, role, rolebinding, clusterrole, clusterrolebinding, service, pdb.",
               "# Create the objects of a manifest\n"
               "kubectl create -f gpu-pod.yaml\n"
               "# Create a namespace\n"
               "kubectl create namespace ml\n"
               "# Create a configmap from literals\n"
               "kubectl create configmap cfg --from-literal=k=v"),
    "apply": ("Apply a configuration to a resource by filename or stdin",
              "Creates the objects that do not exist and updates the others with a three-way merge of the "
              "last-applied configuration, the live object and the new file. --prune deletes objects that were "
              "applied before but are no longer in the files. view-last-applied, set-last-applied and "
              "edit-last-applied work on the stored configuration.",
              "# Apply a manifest\n"
              "kubectl apply -f deploy.yaml\n"
              "# Apply a directory and prune what left it\n"
              "kubectl apply -f manifests/ --prune -l app=web\n"
              "# Show the last applied configuration\n"
              "kubectl apply view-last-applied deployment/web"),
    "delete": ("Delete resources by filenames, stdin, resources and names, or by resources and label selector",
               "Deletes the named objects or every object matching a selector. --grace-period overrides the "
               "pod termination grace period; --cascade=false orphans dependents.",
               "# Delete a pod\n"
               "kubectl delete pod trainer\n"
               "# Delete the objects of a manifest\n"
               "kubectl delete -f gpu-pod.yaml\n"
               "# Delete all pods with a label, immediately\n"
               "kubectl delete pods -l app=train --grace-period=0"),
    "logs": ("Print the logs for a container in a pod",
             "Prints the output of one container of a pod (-c selects it). --tail limits the number of lines; "
             "-w/--follow streams new output.",
             "# Logs of a single-container pod\n"
             "kubectl logs gpu-pod\n"
             "# Last 20 lines of one container\n"
             "kubectl logs trainer -c worker --tail 20"),
    "exec": ("Execute a command in a container",
             "Runs a command inside a running container. -i passes stdin, -t allocates a terminal.",
             "# Run a command in a pod\n"
             "kubectl exec trainer -- rocm-smi\n"
             "# Open an interactive shell\n"
             "kubectl exec -i -t trainer -- sh"),
    "label": ("Update the labels on a resource",
              "Adds, overwrites (--overwrite) or removes (key-) labels of objects.",
              "# Label a node\n"
              "kubectl label node mi355x-0 gpu-pool=train\n"
              "# Remove a label\n"
              "kubectl label pod trainer app-"),
    "annotate": ("Update the annotations on a resource",
                 "Adds, overwrites (--overwrite) or removes (key-) annotations of objects.",
                 "# Annotate a pod\n"
                 "kubectl annotate pod trainer owner=ml-team\n"
                 "# Remove an annotation\n"
                 "kubectl annotate pod trainer owner-"),
    "cordon": ("Mark node as unschedulable",
               "Sets spec.unschedulable on a node so that the scheduler places no new pods on it.",
               "# Stop scheduling onto a node\n"
               "kubectl cordon mi355x-0"),
    "uncordon": ("Mark node as schedulable",
                 "Clears spec.unschedulable on a node.",
                 "# Allow scheduling onto a node again\n"
                 "kubectl uncordon mi355x-0"),
    "drain": ("Drain node in preparation for maintenance",
              "Cordons the node and evicts its pods through the eviction API (honouring disruption budgets). "
              "DaemonSet pods need --ignore-daemonsets; mirror pods are skipped.",
              "# Drain a node before a GPU firmware update\n"
              "kubectl drain mi355x-0 --ignore-daemonsets"),
    "scale": ("Set a new size for a Deployment, ReplicaSet, Replication Controller, or Job",
              "Updates the replica count through the scale subresource.",
              "# Scale a deployment to 4 replicas\n"
              "kubectl scale deployment/web --replicas 4"),
    "patch": ("Update field(s) of a resource using strategic merge patch",
              "Applies a strategic-merge (default), JSON-merge (--type merge) or JSON patch (--type json) to an "
              "object.",
              "# Set a node label with a merge patch\n"
              "kubectl patch node mi355x-0 --type merge -p '{\"metadata\":{\"labels\":{\"a\":\"b\"}}}'"),
    "run": ("Run a particular image on the cluster",
            "Creates a pod (--restart Never) or a deployment running one image. --gpus asks for that many "
            "amd.com/gpu devices.",
            "# Run one vector-add pod on a GPU\n"
            "kubectl run vadd --image rocm/vector-add --restart Never --gpus 1\n"
            "# Run a deployment of 3 replicas\n"
            "kubectl run web --image nginx --replicas 3"),
    "top": ("Display Resource (CPU/Memory/GPU) usage",
            "Shows current CPU and memory use of nodes or pods from the resource metrics API (kubelet "
            "summaries as a fallback), and per-GPU utilisation with `top gpu`.",
            "# Node usage\n"
            "kubectl top node\n"
            "# Pod usage in a namespace\n"
            "kubectl top pod -n ml\n"
            "# GPU usage per device\n"
            "kubectl top gpu"),
    "version": ("Print the client and server version information",
                "Prints the kubectl build and the version the API server reports.",
                "# Client and server versions\n"
                "kubectl version"),
    "api-resources": ("Print the supported API resources on the server",
                      "Lists every resource the server serves with its short names, API group, namespacing "
                      "and kind.",
                      "# All resources\n"
                      "kubectl api-resources"),
    "api-versions": ("Print the supported API versions on the server, in the form of \"group/version\"",
                     "Lists every group/version the discovery endpoints advertise.",
                     "# All group versions\n"
                     "kubectl api-versions"),
    "cluster-info": ("Display cluster info",
                     "Prints the address of the control plane and of the cluster services. `cluster-info "
                     "dump` writes the state of the cluster for debugging.",
                     "# Control plane address\n"
                     "kubectl cluster-info\n"
                     "# Dump cluster state to a directory\n"
                     "kubectl cluster-info dump --output-directory /tmp/state"),
    "wait": ("Wait for a specific condition on one or many resources",
             "Blocks until the objects meet --for (condition=<name> or delete) or --timeout passes.",
             "# Wait until a pod is ready\n"
             "kubectl wait pod/trainer --for condition=Ready --timeout 60\n"
             "# Wait until a pod is gone\n"
             "kubectl wait pod/old --for delete"),
    "attach": ("Attach to a running container",
               "Connects to the output (and with -i the input) of a running container's main process.",
               "# Attach to a pod's output\n"
               "kubectl attach trainer\n"
               "# Attach interactively\n"
               "kubectl attach -i -t trainer"),
    "edit": ("Edit a resource on the server",
             "Opens the object in $KUBE_EDITOR or $EDITOR and updates it with the edited content.",
             "# Edit a deployment\n"
             "kubectl edit deployment/web"),
    "replace": ("Replace a resource by filename or stdin",
                "Replaces whole objects with the content of the files. --force deletes and re-creates.",
                "# Replace a pod's definition\n"
                "kubectl replace -f gpu-pod.yaml"),
    "expose": ("Take a replication controller, service, deployment or pod and expose it as a new Kubernetes Service",
               "Creates a service selecting the pods of the object, with the given port and type.",
               "# Expose a deployment on port 80\n"
               "kubectl expose deployment web --port 80 --target-port 8080"),
    "autoscale": ("Auto-scale a Deployment, ReplicaSet, or ReplicationController",
                  "Creates a horizontal pod autoscaler with the given bounds and CPU (or GPU) target.",
                  "# Keep 2 to 10 replicas at 80% CPU\n"
                  "kubectl autoscale deployment web --min 2 --max 10 --cpu-percent 80"),
    "taint": ("Update the taints on one or more nodes",
              "Adds (key=value:effect), or removes (key:effect- or key-) node taints.",
              "# Reserve a node for GPU jobs\n"
              "kubectl taint node mi355x-0 dedicated=gpu:NoSchedule\n"
              "# Remove the taint\n"
              "kubectl taint node mi355x-0 dedicated:NoSchedule-"),
    "rollout": ("Manage the rollout of a resource",
                "Subcommands status, history, undo, pause and resume for deployments, daemonsets and "
                "statefulsets.",
                "# Watch a rollout\n"
                "kubectl rollout status deployment/web\n"
                "# Roll back to the previous revision\n"
                "kubectl rollout undo deployment/web"),
    "rolling-update": ("Perform a rolling update of the given ReplicationController",
                       "Replaces the pods of a replication controller one by one with those of a new "
                       "controller or image.",
                       "# Update the image of a controller\n"
                       "kubectl rolling-update frontend --image nginx:2"),
    "set": ("Set specific features on objects",
            "Subcommands env, image, resources, selector, serviceaccount and subject change one aspect of "
            "existing objects.",
            "# Change a container image\n"
            "kubectl set image deployment/web web=nginx:2\n"
            "# Set resource limits, including GPUs\n"
            "kubectl set resources deployment/train --limits amd.com/gpu=2"),
    "convert": ("Convert config files between different API versions",
                "Rewrites the objects of the files to another API version (--output-version).",
                "# Convert a file to apps/v1beta2\n"
                "kubectl convert -f deploy.yaml --output-version apps/v1beta2"),
    "completion": ("Output shell completion code for the specified shell (bash or zsh)",
                   "Prints a completion script to source from the shell's startup file.",
                   "# Load bash completion\n"
                   "source <(kubectl completion bash)"),
    "options": ("Print the list of flags inherited by all commands",
                "Lists the global flags every command accepts.",
                "# Global flags\n"
                "kubectl options"),
    "plugin": ("Runs a command-line plugin",
               "Runs an executable plugin found in the plugin directories (~/.kube/plugins and "
               "$KUBECTL_PLUGINS_PATH).",
               "# Run a plugin\n"
               "kubectl plugin hello"),
    "port-forward": ("Forward one or more local ports to a pod",
                     "Listens on local ports and forwards each connection to the pod's port through the "
                     "kubelet streaming server.",
                     "# Forward local 8888 to the pod's 8080\n"
                     "kubectl port-forward trainer 8888:8080"),
    "proxy": ("Run a proxy to the Kubernetes API server",
              "Serves the API server's API on a local port with the client's credentials.",
              "# Proxy the API on port 8001\n"
              "kubectl proxy --port 8001"),
    "cp": ("Copy files and directories to and from containers",
           "Copies with tar through exec: <pod>:<path> on either side.",
           "# Copy a file out of a pod\n"
           "kubectl cp trainer:/out/result.json ./result.json"),
    "explain": ("Documentation of resources",
                "Prints the fields of a resource from the server's OpenAPI document, recursively with "
                "--recursive, for a field path such as pods.spec.extendedResources.",
                "# Fields of a pod\n"
                "kubectl explain pods\n"
                "# The fork's device-granular request field\n"
                "kubectl explain pods.spec.extendedResources"),
    "auth": ("Inspect authorization",
             "`auth can-i` asks the server whether the current user may perform a verb on a resource.",
             "# Check a permission\n"
             "kubectl auth can-i create pods"),
    "certificate": ("Modify certificate resources",
                    "`certificate approve` and `certificate deny` set the condition of certificate signing "
                    "requests.",
                    "# Approve a kubelet's CSR\n"
                    "kubectl certificate approve node-csr-abc"),
    "alpha": ("Commands for features in alpha",
              "`alpha diff` compares LOCAL, LIVE, LAST and MERGED versions of the objects of files.",
              "# Diff a file against the live objects\n"
              "kubectl alpha diff -f deploy.yaml LIVE LOCAL"),
    "config": ("Modify kubeconfig files",
               "Subcommands view, use-context, current-context, get-contexts, get-clusters, set-cluster, "
               "set-credentials, set-context, set, unset, rename-context, delete-context and delete-cluster "
               "edit the kubeconfig file (--kubeconfig, $KUBECONFIG or ~/.kube/config).",
               "# Show the merged configuration\n"
               "kubectl config view\n"
               "# Switch context\n"
               "kubectl config use-context prod"),
    "help": ("Help about any command",
             "Prints the help of a command, or the list of commands.",
             "# List commands\n"
             "kubectl help\n"
             "# Help of one command\n"
             "kubectl help get"),
}


def examples(cmd: str) -> str:
    """The command's examples in the reference's normal form: every line indented by two
    spaces (templates.Examples)."""
    ex = HELP.get(cmd, ("", "", ""))[2]
    return "\n".join(INDENT + line for line in ex.splitlines())


def long_desc(cmd: str) -> str:
    return textwrap.fill(HELP.get(cmd, ("", "", ""))[1], 100).strip()


def short(cmd: str) -> str:
    return HELP.get(cmd, ("", "", ""))[0]


GROUPS = [
    ("Basic Commands (Beginner)", ["create", "expose", "run", "set"]),
    ("Basic Commands (Intermediate)", ["get", "explain", "edit", "delete"]),
    ("Deploy Commands", ["rollout", "rolling-update", "scale", "autoscale"]),
    ("Cluster Management Commands", ["certificate", "cluster-info", "top", "cordon", "uncordon", "drain", "taint"]),
    ("Troubleshooting and Debugging Commands", ["describe", "logs", "attach", "exec", "port-forward", "proxy", "cp",
                                                "auth", "wait"]),
    ("Advanced Commands", ["apply", "patch", "replace", "convert", "alpha"]),
    ("Settings Commands", ["label", "annotate", "completion"]),
    ("Other Commands", ["api-resources", "api-versions", "config", "help", "plugin", "version", "options"]),
]


def overview() -> str:
    """`kubectl` / `kubectl help` text: commands grouped as the reference's root command."""
    out = ["kubectl controls the amdkube cluster manager.", ""]
    seen = set()
    for title, cmds in GROUPS:
        out.append(f"{title}:")
        for c in cmds:
            seen.add(c)
            out.append(f"  {c:<15}{short(c)}")
        out.append("")
    rest = sorted(set(HELP) - seen)
    if rest:
        out.append("Other:")
        out += [f"  {c:<15}{short(c)}" for c in rest]
        out.append("")
    out.append('Use "kubectl <command> --help" for more information about a given command.')
    return "\n".join(out)


def command_help(cmd: str) -> str:
    if cmd not in HELP:
        return f'Unknown help topic "{cmd}"\n\n' + overview()
    return f"{long_desc(cmd)}\n\nExamples:\n{examples(cmd)}\n\nUsage:\n  kubectl {cmd} [flags]"

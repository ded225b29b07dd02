"""Component entry points: `python -m amdkube <component> [flags]`.

Flag names follow the reference binaries (cmd/kube-apiserver/app/options, plugin/cmd/
kube-scheduler/app/server.go:106-160, cmd/kubelet/app/options/options.go,
cmd/kube-controller-manager) where a counterpart exists. `local-up` mirrors
hack/local-up-cluster.sh (:394-784): apiserver → controller-manager → scheduler → rocshim →
device plugin → kubelet as separate processes with logs under --log-dir.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import signal
import socket
import shutil
import subprocess
import sys
import time

from ..utils import log as klog


def _client(a, **kw):
    """--kubeconfig wins over --server (plus the kubelet's --token from TLS bootstrap); a component
    left at the default --server inside a pod uses the in-cluster config (ServiceAccount token,
    cluster CA, KUBERNETES_SERVICE_HOST), as client-go's BuildConfigFromFlags falls back to it."""
    from ..client import Client
    if getattr(a, "kubeconfig", None):
        return Client.from_kubeconfig(a.kubeconfig, **kw)
    if a.server in ("http://127.0.0.1:8080", "", None) and os.environ.get("KUBERNETES_SERVICE_HOST") \
            and not getattr(a, "token", None):
        from ..client.rest import ConfigError
        try:
            return Client.in_cluster(**kw)
        except ConfigError as e:
            logging.getLogger("amdkube").warning("in-cluster config unavailable (%s); using --server %s", e, a.server)
    return Client(a.server, token=getattr(a, "token", None), **kw)


async def _serve_health(component, host: str, port: int, name: str):
    """/healthz and /metrics of a control-plane daemon (the reference's insecure --port)."""
    from aiohttp import web
    from ..utils import profiling
    from ..utils.metrics import CONTENT_TYPE, new_registry, render
    app = web.Application()

    async def healthz(_):
        return web.Response(text="ok")

    async def metrics(_):
        reg = getattr(component, "metrics", None) or new_registry()
        return web.Response(body=render(reg), headers={"Content-Type": CONTENT_TYPE})
    app.router.add_get("/healthz", healthz)
    app.router.add_get("/metrics", metrics)
    profiling.add_routes(app)
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    try:
        await web.TCPSite(runner, host, port, reuse_address=True).start()
    except OSError as e:
        logging.getLogger(f"amdkube.{name}").warning("cannot serve /healthz on %s:%d: %s", host, port, e)
        await runner.cleanup()
        return None
    logging.getLogger(f"amdkube.{name}").info("serving /healthz and /metrics on %s:%d", host, port)
    stop = getattr(component, "stop", None)
    if stop is not None:
        async def stop_all():
            await runner.cleanup()
            await stop()
        component.stop = stop_all
    return runner


def _run_forever(coro_factory):
    async def main():
        stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for s in (signal.SIGINT, signal.SIGTERM):
            loop.add_signal_handler(s, stop.set)
        while True:
            comp = await coro_factory()
            # a component may ask to be rebuilt in place (dynamic kubelet config: the reference
            # kubelet exits for its supervisor to restart it with the new checkpoint)
            restart = getattr(comp, "restart_requested", None) or asyncio.Event()
            done, _ = await asyncio.wait([asyncio.create_task(stop.wait()), asyncio.create_task(restart.wait())],
                                         return_when=asyncio.FIRST_COMPLETED)
            if hasattr(comp, "stop"):
                await comp.stop()
            if stop.is_set():
                return
            logging.getLogger("amdkube").info("restarting %s to apply new configuration", type(comp).__name__)
    prof_path = os.environ.get("AMDKUBE_CPROFILE")   # whole-process profile of a daemon, written on SIGTERM
    if prof_path:
        import cProfile
        pr = cProfile.Profile()
        pr.enable()
        try:
            asyncio.run(main())
        finally:
            pr.disable()
            pr.dump_stats(f"{prof_path}.{os.getpid()}")
        return
    asyncio.run(main())


def apiserver(argv):
    ap = argparse.ArgumentParser("amdkube apiserver")
    ap.add_argument("--bind-address", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080, help="the main listener (TLS when certificates are given)")
    ap.add_argument("--secure-port", type=int, default=None, help="TLS listener (with --tls-cert-file)")
    ap.add_argument("--insecure-port", type=int, default=None,
                    help="unauthenticated listener next to --secure-port (alone: the main listener)")
    ap.add_argument("--insecure-bind-address", default="127.0.0.1")
    ap.add_argument("--data-dir", default=None, help="MVCC store WAL/snapshot directory (etcd replacement)")
    ap.add_argument("--store-conflict-chance", type=float, default=0.0,
                    help="fault injection: share of conditional store writes that fail as a lost race (retried above)")
    ap.add_argument("--data-dir-lock-wait", type=float, default=10.0,
                    help="seconds to wait for another process to release --data-dir (a self-hosted apiserver "
                         "taking over from its static Pod waits for the hand-off)")
    ap.add_argument("--admission-control", default=None, help="ordered, comma-separated admission plugins")
    ap.add_argument("--resource-v2-resources", default="amd.com/gpu", help="container limits ResourceV2 converts")
    ap.add_argument("--token-auth-file", default=None)
    ap.add_argument("--anonymous-auth", default="true")
    ap.add_argument("--authorization-mode", default="AlwaysAllow")
    ap.add_argument("--max-requests-inflight", type=int, default=400)
    ap.add_argument("--max-mutating-requests-inflight", type=int, default=200)
    ap.add_argument("--event-ttl", type=float, default=3600.0)
    ap.add_argument("--service-cluster-ip-range", default="10.0.0.0/24")
    ap.add_argument("--service-node-port-range", default="30000-32767")
    ap.add_argument("--service-account-key-file", default=None, help="HMAC key for service-account tokens")
    ap.add_argument("--tls-cert-file", default=None)
    ap.add_argument("--tls-private-key-file", default=None)
    ap.add_argument("--client-ca-file", default=None)
    ap.add_argument("-v", type=int, default=0)
    ap.add_argument("--audit-log-path", default=None, help="write audit events (JSON lines) here; - for stdout")
    ap.add_argument("--kubelet-https", default="false", choices=("true", "false"))
    ap.add_argument("--kubelet-client-certificate", default=None)
    ap.add_argument("--kubelet-client-key", default=None)
    ap.add_argument("--kubelet-certificate-authority", default=None)
    ap.add_argument("--audit-policy-file", default=None, help="audit.k8s.io Policy (default: everything at Metadata)")
    ap.add_argument("--audit-log-maxsize", type=int, default=0, help="rotate the audit log at this many MB")
    ap.add_argument("--audit-log-maxbackup", type=int, default=0, help="rotated audit logs to keep")
    ap.add_argument("--requestheader-client-ca-file", default=None,
                    help="CA of front-proxy client certs allowed to assert X-Remote-User/Group")
    ap.add_argument("--requestheader-allowed-names", default="", help="front-proxy cert CNs accepted (empty: any)")
    ap.add_argument("--proxy-client-cert-file", default=None, help="aggregator's client cert towards extension apiservers")
    ap.add_argument("--proxy-client-key-file", default=None)
    tf = lambda v: str(v).lower() in ("true", "1", "yes")   # noqa: E731
    lst = lambda v: [x.strip() for x in v.split(",") if x.strip()]   # noqa: E731
    ap.add_argument("--requestheader-username-headers", type=lst, default=["X-Remote-User"])
    ap.add_argument("--requestheader-group-headers", type=lst, default=["X-Remote-Group"])
    ap.add_argument("--requestheader-extra-headers-prefix", type=lst, default=["X-Remote-Extra-"])
    ap.add_argument("--basic-auth-file", default=None)
    ap.add_argument("--oidc-issuer-url", default=None)
    ap.add_argument("--oidc-client-id", default=None)
    ap.add_argument("--oidc-ca-file", default=None)
    ap.add_argument("--oidc-username-claim", default="sub")
    ap.add_argument("--oidc-username-prefix", default=None)
    ap.add_argument("--oidc-groups-claim", default=None)
    ap.add_argument("--oidc-groups-prefix", default="")
    ap.add_argument("--authentication-token-webhook-config-file", default=None)
    ap.add_argument("--authentication-token-webhook-cache-ttl", type=float, default=120.0, help="seconds")
    ap.add_argument("--authorization-policy-file", default=None, help="ABAC policy (one JSON Policy per line)")
    ap.add_argument("--authorization-webhook-config-file", default=None)
    ap.add_argument("--authorization-webhook-cache-authorized-ttl", type=float, default=300.0, help="seconds")
    ap.add_argument("--authorization-webhook-cache-unauthorized-ttl", type=float, default=30.0, help="seconds")
    ap.add_argument("--experimental-encryption-provider-config", default=None, help="EncryptionConfig file")
    ap.add_argument("--audit-log-format", default="json", choices=("json", "legacy"))
    ap.add_argument("--audit-log-maxage", type=int, default=0, help="days to keep rotated audit logs")
    ap.add_argument("--audit-webhook-config-file", default=None)
    ap.add_argument("--audit-webhook-mode", default="batch", choices=("batch", "blocking"))
    ap.add_argument("--audit-webhook-batch-buffer-size", type=int, default=10000)
    ap.add_argument("--audit-webhook-batch-max-size", type=int, default=400)
    ap.add_argument("--audit-webhook-batch-max-wait", type=float, default=30.0)
    ap.add_argument("--audit-webhook-batch-throttle-qps", type=float, default=10.0)
    ap.add_argument("--audit-webhook-batch-throttle-burst", type=int, default=15)
    ap.add_argument("--advertise-address", default=None)
    ap.add_argument("--kubernetes-service-node-port", type=int, default=0)
    ap.add_argument("--allow-privileged", type=tf, default=True)
    ap.add_argument("--runtime-config", default="", help="group/version=true|false, api/all=false, ...")
    ap.add_argument("--cors-allowed-origins", type=lst, default=[])
    ap.add_argument("--enable-logs-handler", type=tf, default=True)
    ap.add_argument("--profiling", type=tf, default=True)
    ap.add_argument("--min-request-timeout", type=float, default=1800.0, help="seconds (watch duration floor)")
    ap.add_argument("--tls-sni-cert-key", action="append", default=[], help="cert,key[:name1,name2] (repeatable)")
    ap.add_argument("--feature-gates", default="")
    ap.add_argument("--storage-media-type", default="application/json",
                    choices=("application/json", "application/vnd.kubernetes.protobuf"),
                    help="encoding of objects in the store (the reference's etcd3 default is protobuf)")
    # accepted for command-line compatibility: etcd and watch-cache tuning of a store this
    # apiserver embeds, SSH tunnels and other knobs with no counterpart here
    ap.add_argument("--etcd-servers", default=None,
                    help="etcd v3 endpoints (amdkube etcd or etcd) shared by several apiservers; unset: the embedded store")
    ap.add_argument("--etcd-cafile", default=None)
    ap.add_argument("--etcd-certfile", default=None)
    ap.add_argument("--etcd-keyfile", default=None)
    ap.add_argument("--apiserver-count", type=int, default=1,
                    help="apiservers sharing the store: the kubernetes endpoints keep every one's address")
    ap.add_argument("--endpoint-reconciler-type", default="master-count", choices=("master-count", "lease", "none"),
                    help="how the kubernetes service endpoints are kept: master-count (--apiserver-count), "
                         "lease (every apiserver renews a lease; endpoints list the live ones), none")
    for flag in ("--etcd-servers-overrides",
                 "--etcd-prefix", "--etcd-quorum-read", "--etcd-compaction-interval", "--storage-backend",
                 "--storage-versions", "--watch-cache", "--watch-cache-sizes",
                 "--default-watch-cache-size", "--deserialization-cache-size", "--target-ram-mb",
                 "--ssh-user", "--ssh-keyfile", "--cert-dir", "--external-hostname",
                 "--public-address-override", "--kubelet-preferred-address-types", "--kubelet-timeout",
                 "--kubelet-read-only-port", "--kubelet-port", "--max-connection-bytes-per-sec",
                 "--http2-max-streams-per-connection", "--repair-malformed-updates", "--delete-collection-workers",
                 "--enable-garbage-collector", "--enable-aggregator-routing", "--enable-swagger-ui", "--contention-profiling",
                 "--master-service-namespace", "--request-timeout", "--tls-ca-file", "--kubeconfig",
                 "--authentication-kubeconfig", "--authorization-kubeconfig", "--authentication-skip-lookup",
                 "--admission-control-config-file", "--enable-bootstrap-token-auth", "--service-account-lookup",
                 "--tls-cipher-suites", "--tls-min-version", "--log-flush-frequency", "--requestheader-extra-headers"):
        ap.add_argument(flag, default=None, help=argparse.SUPPRESS)
    a = ap.parse_args(argv)
    klog.setup(a.v, "apiserver")
    sni = []
    for item in a.tls_sni_cert_key:
        files, _, names = item.partition(":")
        cert, _, key = files.partition(",")
        sni.append((cert, key, [x for x in names.split(",") if x]))
    transformer = None
    if a.experimental_encryption_provider_config:
        from ..apiserver.encryption import load as load_encryption
        transformer = load_encryption(a.experimental_encryption_provider_config)
    options = {k: getattr(a, k) for k in (
        "requestheader_username_headers", "requestheader_group_headers", "requestheader_extra_headers_prefix",
        "basic_auth_file", "oidc_issuer_url", "oidc_client_id", "oidc_ca_file", "oidc_username_claim",
        "oidc_username_prefix", "oidc_groups_claim", "oidc_groups_prefix", "authentication_token_webhook_config_file",
        "authentication_token_webhook_cache_ttl", "authorization_policy_file", "authorization_webhook_config_file",
        "authorization_webhook_cache_authorized_ttl", "authorization_webhook_cache_unauthorized_ttl",
        "audit_log_format", "audit_log_maxage", "audit_webhook_config_file", "audit_webhook_mode",
        "audit_webhook_batch_buffer_size", "audit_webhook_batch_max_size", "audit_webhook_batch_max_wait",
        "audit_webhook_batch_throttle_qps", "audit_webhook_batch_throttle_burst", "advertise_address",
        "kubernetes_service_node_port", "allow_privileged", "runtime_config", "cors_allowed_origins",
        "enable_logs_handler", "profiling", "min_request_timeout", "storage_media_type", "apiserver_count",
        "endpoint_reconciler_type")}
    options["tls_sni_cert_key"] = sni
    main_port = a.port
    if a.secure_port is not None and a.tls_cert_file:
        main_port = a.secure_port
        options.update(insecure_port=a.insecure_port, insecure_bind_address=a.insecure_bind_address)
    elif a.insecure_port is not None:
        main_port = a.insecure_port
    from ..apiserver import APIServer
    from ..apiserver.admission import DEFAULT_CHAIN
    from ..store import MVCCStore
    tokens = {}
    if a.token_auth_file:
        for line in open(a.token_auth_file):
            parts = [p.strip().strip('"') for p in line.strip().split(",")]
            if len(parts) >= 2:
                tokens[parts[0]] = {"name": parts[1], "uid": parts[2] if len(parts) > 2 else parts[1],
                                    "groups": parts[3].split(",") if len(parts) > 3 else []}

    async def mk():
        if a.etcd_servers:
            from ..store.etcd3 import Etcd3Store
            store = await asyncio.to_thread(Etcd3Store, a.etcd_servers, ca=a.etcd_cafile, cert=a.etcd_certfile,
                                            key=a.etcd_keyfile, transformer=transformer)
        else:
            store = await asyncio.to_thread(MVCCStore, a.data_dir, transformer=transformer, lock_wait=a.data_dir_lock_wait)
        store.conflict_chance = a.store_conflict_chance
        srv = APIServer(store, admission_plugins=(a.admission_control.split(",") if a.admission_control else DEFAULT_CHAIN),
                        admission_config={"ResourceV2": {"resource_names": tuple(a.resource_v2_resources.split(","))}},
                        token_auth=tokens, authorization_mode=a.authorization_mode, anonymous_auth=a.anonymous_auth == "true",
                        max_in_flight=a.max_requests_inflight, max_mutating_in_flight=a.max_mutating_requests_inflight,
                        event_ttl=a.event_ttl, service_cidr=a.service_cluster_ip_range,
                        node_port_range=a.service_node_port_range,
                        service_account_key=open(a.service_account_key_file, "rb").read().strip() if a.service_account_key_file else None,
                        tls_cert_file=a.tls_cert_file, tls_key_file=a.tls_private_key_file, client_ca_file=a.client_ca_file,
                        audit_log_path=a.audit_log_path, audit_policy_file=a.audit_policy_file,
                        audit_log_maxsize=a.audit_log_maxsize, audit_log_maxbackup=a.audit_log_maxbackup,
                        kubelet_https=a.kubelet_https == "true", kubelet_client_certificate=a.kubelet_client_certificate,
                        kubelet_client_key=a.kubelet_client_key, kubelet_certificate_authority=a.kubelet_certificate_authority,
                        requestheader_client_ca_file=a.requestheader_client_ca_file,
                        requestheader_allowed_names=[x for x in a.requestheader_allowed_names.split(",") if x],
                        proxy_client_cert_file=a.proxy_client_cert_file, proxy_client_key_file=a.proxy_client_key_file,
                        options=options)
        return await srv.start(a.bind_address, main_port)
    _run_forever(mk)


def etcd(argv):
    """The etcd v3 API over amdkube's MVCC store (store/etcdserver.py), for apiservers that share
    one store via --etcd-servers."""
    ap = argparse.ArgumentParser("amdkube etcd")
    ap.add_argument("--listen-client-urls", default="http://127.0.0.1:2379")
    ap.add_argument("--data-dir", default=None, help="WAL + snapshot directory (default: memory only)")
    ap.add_argument("--cert-file", default=None)
    ap.add_argument("--key-file", default=None)
    ap.add_argument("--trusted-ca-file", default=None, help="require client certificates signed by this CA")
    ap.add_argument("--snapshot-count", type=int, default=50_000, help="WAL records between snapshots")
    ap.add_argument("--name", default="default", help="this member's name in --initial-cluster")
    ap.add_argument("--initial-cluster", default="",
                    help="name=peerURL,... of every member: a raft group (static membership)")
    ap.add_argument("--listen-peer-urls", default=None, help="raft + member-to-member calls only (default: this "
                                                              "member's --initial-cluster URL)")
    ap.add_argument("--peer-cert-file", default=None, help="peer listener + peer channels: mutual TLS")
    ap.add_argument("--peer-key-file", default=None)
    ap.add_argument("--peer-trusted-ca-file", default=None, help="require peer certificates signed by this CA")
    ap.add_argument("--heartbeat-interval", type=int, default=100, help="ms")
    ap.add_argument("--election-timeout", type=int, default=1000, help="ms")
    ap.add_argument("--client-wire-port", type=int, default=0,
                    help="port of the framed client lane next to the gRPC API (0: any free port, -1: off); "
                         "advertised to clients in Status metadata")
    ap.add_argument("--max-txn-ops", type=int, default=128, help="most compares / success / failure ops in one Txn")
    ap.add_argument("--max-request-bytes", type=int, default=3 * 512 * 1024, help="largest client request accepted")
    ap.add_argument("-v", type=int, default=0)
    for flag in ("--advertise-client-urls", "--initial-advertise-peer-urls", "--initial-cluster-state",
                 "--initial-cluster-token", "--client-cert-auth", "--quota-backend-bytes"):
        ap.add_argument(flag, default=None, help=argparse.SUPPRESS)
    a = ap.parse_args(argv)
    klog.setup(a.v, "etcd")
    from ..store.etcdserver import serve
    strip = lambda u: u.split("://", 1)[-1].rstrip("/")   # noqa: E731
    listen = strip(a.listen_client_urls.split(",")[0])
    peers = {}
    for item in filter(None, a.initial_cluster.split(",")):
        n, _, url = item.partition("=")
        peers[n.strip()] = strip(url)
    if peers and a.name not in peers:
        ap.error(f"--name {a.name} is not in --initial-cluster")
    peer_listen = strip(a.listen_peer_urls.split(",")[0]) if a.listen_peer_urls else peers.get(a.name)
    coro = serve(a.data_dir, listen, a.cert_file, a.key_file, a.trusted_ca_file, a.snapshot_count,
                 name=a.name, peers=peers, peer_listen=peer_listen,
                 heartbeat=a.heartbeat_interval / 1000.0, election=a.election_timeout / 1000.0,
                 peer_cert=a.peer_cert_file, peer_key=a.peer_key_file, peer_ca=a.peer_trusted_ca_file,
                 wire_port=a.client_wire_port, max_txn_ops=a.max_txn_ops, max_request_bytes=a.max_request_bytes)
    prof_path = os.environ.get("AMDKUBE_CPROFILE")
    pr = None
    if prof_path:
        import cProfile
        pr = cProfile.Profile()
        pr.enable()
        signal.signal(signal.SIGTERM, lambda *_: (_ for _ in ()).throw(KeyboardInterrupt()))
    try:
        asyncio.run(coro)
    except KeyboardInterrupt:
        pass
    finally:
        if pr is not None:
            pr.disable()
            pr.dump_stats(f"{prof_path}.{a.name}.{os.getpid()}")


def scheduler(argv):
    ap = argparse.ArgumentParser("amdkube scheduler")
    ap.add_argument("--master", "--server", dest="server", default="http://127.0.0.1:8080")
    ap.add_argument("--kubeconfig", default=None, help="kubeconfig with the server, CA and credentials")
    ap.add_argument("--token", default=None, help="bearer token for the apiserver")
    ap.add_argument("--policy-config-file", default=None)
    ap.add_argument("--algorithm-provider", default="DefaultProvider")
    ap.add_argument("--scheduler-name", default="default-scheduler")
    ap.add_argument("--leader-elect", default="false")
    ap.add_argument("--port", type=int, default=10251)
    ap.add_argument("--feature-gates", default="")
    ap.add_argument("--kube-api-qps", type=float, default=0)
    ap.add_argument("--disable-preemption", action="store_true")
    ap.add_argument("--config", default=None, help="KubeSchedulerConfiguration file (overrides the flags it sets)")
    ap.add_argument("--address", default="127.0.0.1", help="healthz/metrics listener address")
    ap.add_argument("--policy-configmap", default=None, help="ConfigMap whose policy.cfg holds the Policy")
    ap.add_argument("--policy-configmap-namespace", default="kube-system")
    ap.add_argument("--use-legacy-policy-config", default="false", choices=("true", "false"),
                    help="true: --policy-config-file only, never --policy-configmap")
    ap.add_argument("--hard-pod-affinity-symmetric-weight", type=int, default=1)
    ap.add_argument("--lock-object-name", default="kube-scheduler")
    ap.add_argument("--lock-object-namespace", default="kube-system")
    ap.add_argument("--kube-api-burst", type=int, default=0)
    for flag in ("--kube-api-content-type", "--failure-domains", "--profiling", "--contention-profiling"):
        ap.add_argument(flag, default=None, help=argparse.SUPPRESS)
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "scheduler")
    if a.config:     # componentconfig KubeSchedulerConfiguration
        import yaml
        cfg = yaml.safe_load(open(a.config)) or {}
        a.scheduler_name = cfg.get("schedulerName", a.scheduler_name)
        src = cfg.get("algorithmSource") or {}
        if src.get("provider"):
            a.algorithm_provider = src["provider"]
        pol = src.get("policy") or {}
        if (pol.get("file") or {}).get("path"):
            a.policy_config_file = pol["file"]["path"]
        if pol.get("configMap"):
            a.policy_configmap = pol["configMap"].get("name")
            a.policy_configmap_namespace = pol["configMap"].get("namespace", a.policy_configmap_namespace)
        a.hard_pod_affinity_symmetric_weight = int(cfg.get("hardPodAffinitySymmetricWeight", a.hard_pod_affinity_symmetric_weight))
        le = cfg.get("leaderElection") or {}
        if "leaderElect" in le:
            a.leader_elect = "true" if le["leaderElect"] else "false"
        a.lock_object_name = le.get("lockObjectName", a.lock_object_name)
        a.lock_object_namespace = le.get("lockObjectNamespace", a.lock_object_namespace)
        cc = cfg.get("clientConnection") or {}
        a.kubeconfig = cc.get("kubeconfig") or a.kubeconfig
        a.kube_api_qps = float(cc.get("qps", a.kube_api_qps))
        a.kube_api_burst = int(cc.get("burst", a.kube_api_burst))
        if cfg.get("healthzBindAddress"):
            host, _, port = cfg["healthzBindAddress"].rpartition(":")
            a.address, a.port = host or a.address, int(port)
        a.disable_preemption = bool(cfg.get("disablePreemption", a.disable_preemption))
    from ..client import Client
    from ..scheduler import Scheduler
    cm = None
    if a.policy_configmap and a.use_legacy_policy_config != "true" and not a.policy_config_file:
        cm = (a.policy_configmap_namespace, a.policy_configmap)

    async def mk():
        return await Scheduler(_client(a, qps=a.kube_api_qps, burst=a.kube_api_burst), a.scheduler_name,
                               a.policy_config_file, a.algorithm_provider, a.feature_gates, a.leader_elect == "true",
                               port=a.port or None, disable_preemption=a.disable_preemption,
                               hard_pod_affinity_weight=a.hard_pod_affinity_symmetric_weight,
                               lock_object_name=a.lock_object_name, lock_object_namespace=a.lock_object_namespace,
                               address=a.address, policy_configmap=cm).start()
    _run_forever(mk)


def controller_manager(argv):
    ap = argparse.ArgumentParser("amdkube controller-manager")
    ap.add_argument("--master", "--server", dest="server", default="http://127.0.0.1:8080")
    ap.add_argument("--kubeconfig", default=None, help="kubeconfig with the server, CA and credentials")
    ap.add_argument("--token", default=None, help="bearer token for the apiserver")
    ap.add_argument("--controllers", default="*", help="'*' = defaults; 'name' enables, '-name' disables")
    ap.add_argument("--leader-elect", default="false")
    ap.add_argument("--node-monitor-grace-period", type=float, default=40.0)
    ap.add_argument("--pod-eviction-timeout", type=float, default=300.0)
    ap.add_argument("--allocate-node-cidrs", default="false")
    ap.add_argument("--cluster-cidr", default="10.244.0.0/16")
    ap.add_argument("--node-cidr-mask-size", type=int, default=24)
    ap.add_argument("--cloud-provider", default="")
    ap.add_argument("--cloud-config", default=None, help="JSON/YAML provider config (baremetal: loadBalancerIPRange, zone)")
    ap.add_argument("--configure-cloud-routes", default="true")
    ap.add_argument("--cluster-name", default="kubernetes")
    ap.add_argument("--service-account-private-key-file", default=None)
    ap.add_argument("--root-ca-file", default=None)
    ap.add_argument("--cluster-signing-cert-file", default=None)
    ap.add_argument("--cluster-signing-key-file", default=None)
    ap.add_argument("--horizontal-pod-autoscaler-sync-period", type=float, default=30.0)
    ap.add_argument("--horizontal-pod-autoscaler-upscale-delay", type=float, default=180.0)
    ap.add_argument("--horizontal-pod-autoscaler-downscale-delay", type=float, default=300.0)
    ap.add_argument("--hostpath-pv-root", default="/var/lib/amdkube/hostpath-pv")
    ap.add_argument("--node-monitor-period", type=float, default=5.0)
    ap.add_argument("--node-startup-grace-period", type=float, default=60.0)
    ap.add_argument("--node-eviction-rate", type=float, default=0.1)
    ap.add_argument("--secondary-node-eviction-rate", type=float, default=0.01)
    ap.add_argument("--unhealthy-zone-threshold", type=float, default=0.55)
    ap.add_argument("--large-cluster-size-threshold", type=int, default=50)
    ap.add_argument("--enable-taint-manager", default="true", choices=("true", "false"))
    ap.add_argument("--terminated-pod-gc-threshold", type=int, default=12500)
    ap.add_argument("--feature-gates", default="", help="TaintBasedEvictions=false selects the legacy pod-deletion path")
    ap.add_argument("--kube-api-qps", type=float, default=20.0)
    ap.add_argument("--kube-api-burst", type=int, default=30)
    ap.add_argument("--address", default="127.0.0.1", help="healthz/metrics listener")
    ap.add_argument("--port", type=int, default=10252, help="healthz/metrics port (0: off)")
    # accepted for command-line compatibility; this controller manager has no such knob
    for flag in ("--concurrent-deployment-syncs", "--concurrent-endpoint-syncs", "--concurrent-gc-syncs",
                 "--concurrent-namespace-syncs", "--concurrent-replicaset-syncs", "--concurrent-resource-quota-syncs",
                 "--concurrent-service-syncs", "--concurrent-serviceaccount-token-syncs", "--concurrent-rc-syncs",
                 "--deployment-controller-sync-period", "--namespace-sync-period", "--pvclaimbinder-sync-period",
                 "--resource-quota-sync-period", "--route-reconciliation-period", "--node-sync-period", "--service-sync-period",
                 "--min-resync-period", "--controller-start-interval", "--attach-detach-reconcile-sync-period",
                 "--disable-attach-detach-reconcile-sync", "--horizontal-pod-autoscaler-tolerance",
                 "--horizontal-pod-autoscaler-use-rest-clients", "--experimental-cluster-signing-duration",
                 "--enable-dynamic-provisioning", "--enable-hostpath-provisioner", "--flex-volume-plugin-dir",
                 "--use-service-account-credentials", "--service-cluster-ip-range", "--cidr-allocator-type",
                 "--allow-untagged-cloud", "--deleting-pods-qps", "--deleting-pods-burst", "--register-retry-count",
                 "--kube-api-content-type", "--profiling", "--contention-profiling", "--enable-garbage-collector",
                 "--insecure-experimental-approve-all-kubelet-csrs-for-group", "--pv-recycler-increment-timeout-nfs",
                 "--pv-recycler-minimum-timeout-hostpath", "--pv-recycler-minimum-timeout-nfs",
                 "--pv-recycler-pod-template-filepath-hostpath", "--pv-recycler-pod-template-filepath-nfs",
                 "--pv-recycler-timeout-increment-hostpath"):
        ap.add_argument(flag, default=None, help=argparse.SUPPRESS)
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "controller-manager")
    import yaml
    from ..client import Client
    from ..cloudprovider import get_cloud_provider
    from ..controllers import ControllerManager, Options, resolve_controllers
    from ..cloudprovider import load_config as _load_cloud_config
    cfg = _load_cloud_config(a.cloud_config)
    rd = lambda p: open(p, "rb").read().strip() if p else None  # noqa: E731
    opts = Options(node_monitor_grace=a.node_monitor_grace_period, pod_eviction_timeout=a.pod_eviction_timeout,
                   cluster_cidr=a.cluster_cidr, node_cidr_mask_size=a.node_cidr_mask_size,
                   allocate_node_cidrs=a.allocate_node_cidrs == "true", configure_cloud_routes=a.configure_cloud_routes == "true",
                   cloud=get_cloud_provider(a.cloud_provider, cfg), cluster_name=a.cluster_name,
                   service_account_key=rd(a.service_account_private_key_file), root_ca=rd(a.root_ca_file) or b"",
                   cluster_signing_cert_file=a.cluster_signing_cert_file, cluster_signing_key_file=a.cluster_signing_key_file,
                   hostpath_pv_root=a.hostpath_pv_root, hpa_sync_period=a.horizontal_pod_autoscaler_sync_period,
                   hpa_upscale_delay=a.horizontal_pod_autoscaler_upscale_delay,
                   hpa_downscale_delay=a.horizontal_pod_autoscaler_downscale_delay,
                   node_monitor_period=a.node_monitor_period, node_startup_grace=a.node_startup_grace_period,
                   node_eviction_rate=a.node_eviction_rate, secondary_node_eviction_rate=a.secondary_node_eviction_rate,
                   unhealthy_zone_threshold=a.unhealthy_zone_threshold,
                   large_cluster_size_threshold=a.large_cluster_size_threshold,
                   enable_taint_manager=a.enable_taint_manager == "true",
                   terminated_pod_gc_threshold=a.terminated_pod_gc_threshold,
                   taint_based_evictions="TaintBasedEvictions=false" not in a.feature_gates.replace(" ", ""))
    names = resolve_controllers(a.controllers, opts)

    async def mk():
        cm = await ControllerManager(_client(a, qps=a.kube_api_qps, burst=a.kube_api_burst), names,
                                     a.leader_elect == "true", socket.gethostname(), options=opts).start()
        if a.port:
            await _serve_health(cm, a.address, a.port, "kube-controller-manager")
        return cm
    _run_forever(mk)


def cloud_controller_manager(argv):
    """cmd/cloud-controller-manager: the cloud-specific control loops (cloud-node, service,
    route, persistentvolume-labeler) split out of kube-controller-manager; kubelets run with
    --cloud-provider=external and wait, tainted, to be initialised by it."""
    ap = argparse.ArgumentParser("amdkube cloud-controller-manager")
    ap.add_argument("--master", "--server", dest="server", default="http://127.0.0.1:8080")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--token", default=None)
    ap.add_argument("--cloud-provider", required=True, help="aws | gce | azure | openstack | vsphere | cloudstack | ovirt | photon | baremetal | fake")
    ap.add_argument("--cloud-config", default=None, help="provider config (baremetal: loadBalancerIPRange, zone, region, "
                                                         "instances inventory)")
    ap.add_argument("--controllers", default="*", help="'*' = cloud-node,service,route,persistentvolume-labeler")
    ap.add_argument("--allocate-node-cidrs", default="false")
    ap.add_argument("--configure-cloud-routes", default="true")
    ap.add_argument("--cluster-name", default="kubernetes")
    ap.add_argument("--node-status-update-frequency", type=float, default=300.0)
    ap.add_argument("--node-monitor-period", type=float, default=5.0)
    ap.add_argument("--leader-elect", default="false")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "cloud-controller-manager")
    import yaml
    from ..cloudprovider import get_cloud_provider
    from ..controllers import CLOUD_CONTROLLERS, ControllerManager, Options
    from ..cloudprovider import load_config as _load_cloud_config
    cfg = _load_cloud_config(a.cloud_config)
    opts = Options(cloud=get_cloud_provider(a.cloud_provider, cfg), cluster_name=a.cluster_name,
                   allocate_node_cidrs=a.allocate_node_cidrs == "true", configure_cloud_routes=a.configure_cloud_routes == "true",
                   extra={"node_status_update_frequency": a.node_status_update_frequency,
                          "node_monitor_period": a.node_monitor_period})
    names = []
    for it in [x.strip() for x in a.controllers.split(",") if x.strip()]:
        if it == "*":
            names += [n for n in CLOUD_CONTROLLERS if n != "route" or (opts.allocate_node_cidrs and opts.configure_cloud_routes)]
        elif it.startswith("-"):
            names = [n for n in names if n != it[1:]]
        elif it in CLOUD_CONTROLLERS:
            names.append(it)
        else:
            raise SystemExit(f"unknown cloud controller {it!r} (have: {', '.join(CLOUD_CONTROLLERS)})")

    async def mk():
        return await ControllerManager(_client(a), names, a.leader_elect == "true", socket.gethostname(), options=opts).start()
    _run_forever(mk)


def gke_certificates_controller(argv):
    """cmd/gke-certificates-controller: signs approved CSRs through an external signing webhook
    (the kubeconfig of --cluster-signing-gke-kubeconfig) instead of a local CA key, optionally
    approving every kubelet client CSR of one group."""
    ap = argparse.ArgumentParser("amdkube gke-certificates-controller")
    ap.add_argument("--master", "--server", dest="server", default="http://127.0.0.1:8080")
    ap.add_argument("--kubeconfig", default=None, help="kubeconfig with authorization and master location information")
    ap.add_argument("--token", default=None)
    ap.add_argument("--cluster-signing-gke-kubeconfig", required=True,
                    help="kubeconfig of the signing service certificates are POSTed to")
    ap.add_argument("--cluster-signing-gke-retry-backoff", type=float, default=0.5,
                    help="initial backoff (s) between signing attempts; later attempts double it")
    ap.add_argument("--insecure-experimental-approve-all-kubelet-csrs-for-group", default="",
                    help="auto-approve every kubelet client CSR from members of this group")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "gke-certificates-controller")
    from ..controllers import ControllerManager, Options
    opts = Options(extra={"signing_kubeconfig": a.cluster_signing_gke_kubeconfig,
                          "signing_retry_backoff": a.cluster_signing_gke_retry_backoff,
                          "approve_group": a.insecure_experimental_approve_all_kubelet_csrs_for_group})
    names = ["csrsigning-webhook"] + (["csrapproving-group"] if a.insecure_experimental_approve_all_kubelet_csrs_for_group else [])

    async def mk():
        return await ControllerManager(_client(a), names, False, socket.gethostname(), options=opts).start()
    _run_forever(mk)


def rktshim(argv):
    """CRI over rkt (pkg/kubelet/rkt, pkg/kubelet/rktshim): point the kubelet's
    --container-runtime-endpoint at --listen to run pods as rkt pods."""
    ap = argparse.ArgumentParser("amdkube rktshim")
    ap.add_argument("--listen", default="/var/run/amdkube/rktshim.sock")
    ap.add_argument("--state-dir", default="/var/lib/amdkube/rktshim")
    ap.add_argument("--rkt-path", default="rkt", help="the rkt binary (with any global flags, e.g. '--dir=…')")
    ap.add_argument("--insecure-options", default="image", help="rkt fetch --insecure-options")
    ap.add_argument("--node-ip", default="127.0.0.1")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "rktshim")
    from ..runtime.rktshim import RktShim

    async def mk():
        return await RktShim(a.listen, a.state_dir, rkt=a.rkt_path, insecure_options=a.insecure_options, node_ip=a.node_ip).start()
    _run_forever(mk)


def kubelet(argv):
    ap = argparse.ArgumentParser("amdkube kubelet")
    ap.add_argument("--api-servers", "--server", dest="server", default="http://127.0.0.1:8080")
    ap.add_argument("--kubeconfig", default=None, help="kubeconfig with the server, CA and credentials")
    ap.add_argument("--token", default=None, help="bearer token for the apiserver")
    ap.add_argument("--hostname-override", "--node-name", dest="node_name", default=socket.gethostname())
    ap.add_argument("--root-dir", default="/var/lib/kubelet")
    ap.add_argument("--device-plugin-dir", default=None)
    ap.add_argument("--device-plugin-v1beta1-socket", default=None)
    ap.add_argument("--container-runtime-endpoint", default="/var/run/amdkube/rocshim.sock")
    ap.add_argument("--address", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=10250)
    ap.add_argument("--runonce", action="store_true", help="run the static pods once, report, and exit (no API server)")
    ap.add_argument("--cloud-provider", default="", help="'external': the cloud-controller-manager initialises the node; "
                                                          "aws | gce | azure | openstack | vsphere | cloudstack | ovirt | photon | baremetal: in-tree (addresses, providerID, zone)")
    ap.add_argument("--cloud-config", default="", help="the in-tree provider's config (cloud.conf INI or YAML)")
    ap.add_argument("--volume-plugin-dir", default=None, help="FlexVolume driver directory")
    ap.add_argument("--enable-controller-attach-detach", default="true", choices=("true", "false"))
    ap.add_argument("--node-ip", default="127.0.0.1")
    ap.add_argument("--node-status-update-frequency", type=float, default=10.0)
    ap.add_argument("--pleg-relist-period", type=float, default=1.0)
    ap.add_argument("--prioritize-device-pods", default="true", choices=("true", "false"),
                    help="start pods that hold accelerators before the other pods of a burst")
    ap.add_argument("--max-pods", type=int, default=110)
    ap.add_argument("--maximum-dead-containers-per-container", type=int, default=1)
    ap.add_argument("--maximum-dead-containers", type=int, default=-1)
    ap.add_argument("--eviction-hard", default=None, help="e.g. memory.available<100Mi,nodefs.available<10%%")
    ap.add_argument("--eviction-soft", default="")
    ap.add_argument("--eviction-soft-grace-period", default="")
    ap.add_argument("--eviction-minimum-reclaim", default="")
    ap.add_argument("--eviction-pressure-transition-period", type=float, default=300.0, help="seconds")
    ap.add_argument("--eviction-max-pod-grace-period", type=int, default=0)
    ap.add_argument("--minimum-container-ttl-duration", type=float, default=0.0, help="seconds")
    ap.add_argument("--node-labels", default="")
    ap.add_argument("--register-with-taints", default="")
    ap.add_argument("--feature-gates", default="")
    ap.add_argument("--chaos-chance", type=float, default=0.0)
    ap.add_argument("--pod-manifest-path", default=None, help="directory of static pod manifests")
    ap.add_argument("--cluster-dns", default="", help="comma-separated DNS server IPs for ClusterFirst pods")
    ap.add_argument("--cluster-domain", default="", help="cluster DNS domain (e.g. cluster.local)")
    ap.add_argument("--resolv-conf", default="/etc/resolv.conf", help="resolver file used as the base of pod DNS")
    ap.add_argument("--file-check-frequency", type=float, default=20.0)
    ap.add_argument("--gpu-stats-backend", default="auto")
    ap.add_argument("--kube-api-qps", type=float, default=0)
    ap.add_argument("--kube-reserved", default="", help="e.g. cpu=500m,memory=1Gi")
    ap.add_argument("--system-reserved", default="", help="e.g. cpu=500m,memory=1Gi")
    ap.add_argument("--enforce-node-allocatable", default="pods")
    ap.add_argument("--cgroup-root", default="", help="cgroup v2 directory of the kubepods hierarchy")
    ap.add_argument("--experimental-allowed-unsafe-sysctls", default="", help="comma-separated sysctls or patterns ending in *")
    ap.add_argument("--cpu-manager-policy", default="none", choices=("none", "static"))
    ap.add_argument("--cpu-manager-reconcile-period", type=float, default=10.0, help="seconds")
    ap.add_argument("--config", default=None, help="KubeletConfiguration file (KubeletConfigFile gate)")
    ap.add_argument("--tls-cert-file", default=None)
    ap.add_argument("--tls-private-key-file", default=None)
    ap.add_argument("--client-ca-file", default=None)
    ap.add_argument("--anonymous-auth", default="true", choices=("true", "false"))
    ap.add_argument("--authentication-token-webhook", action="store_true")
    ap.add_argument("--authorization-mode", default="AlwaysAllow", choices=("AlwaysAllow", "Webhook"))
    ap.add_argument("--cert-dir", default=None)
    ap.add_argument("--rotate-certificates", action="store_true")
    ap.add_argument("--rotate-server-certificates", action="store_true")
    ap.add_argument("--dynamic-config-dir", default=None, help="checkpoints of Node.spec.configSource (DynamicKubeletConfig gate)")
    ap.add_argument("--image-gc-high-threshold", type=int, default=85)
    ap.add_argument("--image-gc-low-threshold", type=int, default=80)
    ap.add_argument("--minimum-image-ttl-duration", type=float, default=120.0, help="seconds")
    tf = lambda s: str(s).lower() in ("true", "1", "yes")   # noqa: E731
    srcs = lambda s: [x.strip() for x in s.split(",") if x.strip()]   # noqa: E731
    ap.add_argument("--bootstrap-kubeconfig", "--experimental-bootstrap-kubeconfig", dest="bootstrap_kubeconfig", default=None,
                    help="token kubeconfig used to obtain a client certificate when --kubeconfig does not exist")
    ap.add_argument("--enable-server", type=tf, default=True)
    ap.add_argument("--enable-debugging-handlers", type=tf, default=True)
    ap.add_argument("--read-only-port", type=int, default=10255, help="0 disables")
    ap.add_argument("--healthz-port", type=int, default=10248, help="0 disables")
    ap.add_argument("--healthz-bind-address", default="127.0.0.1")
    ap.add_argument("--manifest-url", default=None)
    ap.add_argument("--manifest-url-header", default="", help="comma-separated key:value headers")
    ap.add_argument("--http-check-frequency", type=float, default=20.0, help="seconds")
    ap.add_argument("--sync-frequency", type=float, default=60.0, help="seconds")
    ap.add_argument("--register-node", type=tf, default=True)
    ap.add_argument("--register-schedulable", type=tf, default=True)
    ap.add_argument("--pod-cidr", default="")
    ap.add_argument("--provider-id", default="")
    ap.add_argument("--allow-privileged", type=tf, default=True)
    ap.add_argument("--host-network-sources", type=srcs, default=["*"])
    ap.add_argument("--host-pid-sources", type=srcs, default=["*"])
    ap.add_argument("--host-ipc-sources", type=srcs, default=["*"])
    ap.add_argument("--pods-per-core", type=int, default=0)
    ap.add_argument("--serialize-image-pulls", type=tf, default=True)
    ap.add_argument("--registry-qps", type=float, default=5.0)
    ap.add_argument("--registry-burst", type=int, default=10)
    ap.add_argument("--event-qps", type=float, default=5.0)
    ap.add_argument("--event-burst", type=int, default=10)
    ap.add_argument("--kube-api-burst", type=int, default=10)
    ap.add_argument("--kube-api-content-type", default="application/json", help="only JSON is spoken")
    ap.add_argument("--runtime-request-timeout", type=float, default=120.0, help="seconds")
    ap.add_argument("--image-service-endpoint", default=None)
    ap.add_argument("--keep-terminated-pod-volumes", type=tf, default=False)
    ap.add_argument("--volume-stats-agg-period", type=float, default=60.0, help="seconds")
    ap.add_argument("--cpu-cfs-quota", type=tf, default=True)
    ap.add_argument("--protect-kernel-defaults", type=tf, default=False)
    ap.add_argument("--fail-swap-on", "--experimental-fail-swap-on", dest="fail_swap_on", type=tf, default=True)
    ap.add_argument("--oom-score-adj", type=int, default=-999)
    ap.add_argument("--max-open-files", type=int, default=1000000)
    ap.add_argument("--lock-file", default=None)
    ap.add_argument("--exit-on-lock-contention", action="store_true")
    ap.add_argument("--seccomp-profile-root", default=None, help="directory of localhost/<name> seccomp profiles")
    ap.add_argument("--cgroup-driver", default="cgroupfs", choices=("cgroupfs", "systemd"))
    ap.add_argument("--cgroups-per-qos", type=tf, default=True)
    ap.add_argument("--bootstrap-checkpoint-path", default=None,
                    help="directory for checkpoints of pods annotated node.kubernetes.io/bootstrap-checkpoint=true")
    # accepted for command-line compatibility; the settings they tune do not exist on this runtime
    for flag in ("--cadvisor-port", "--containerized", "--hairpin-mode", "--non-masquerade-cidr", "--iptables-masquerade-bit",
                 "--iptables-drop-bit", "--make-iptables-util-chains", "--kubelet-cgroups", "--system-cgroups",
                 "--kube-reserved-cgroup", "--system-reserved-cgroup", "--experimental-qos-reserved",
                 "--streaming-connection-idle-timeout", "--master-service-namespace", "--require-kubeconfig",
                 "--init-config-dir", "--experimental-mounter-path",
                 "--experimental-check-node-capabilities-before-mount", "--experimental-kernel-memcg-notification",
                 "--experimental-allocatable-ignore-eviction", "--enable-custom-metrics", "--contention-profiling",
                 "--really-crash-for-testing", "--authentication-token-webhook-cache-ttl",
                 "--authorization-webhook-cache-authorized-ttl", "--authorization-webhook-cache-unauthorized-ttl"):
        ap.add_argument(flag, default=None, help=argparse.SUPPRESS)
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "kubelet")
    if a.cgroup_driver == "systemd":
        from ..kubelet.cgroups import use_systemd
        if not (use_systemd() or os.environ.get("AMDKUBE_SYSTEMD_BUS")):
            # cgroup_manager_linux.go newManager: "systemd cgroup manager not available"
            raise SystemExit("kubelet: --cgroup-driver=systemd: systemd cgroup manager not available "
                             "(systemd is not the init system of this node)")
    from ..kubelet import node_setup
    lock = node_setup.acquire_lock(a.lock_file, a.exit_on_lock_contention,
                                   on_contention=lambda: os._exit(0)) if a.lock_file else None   # noqa: F841
    if a.fail_swap_on and not a.runonce:
        node_setup.check_swap()
    node_setup.apply_oom_score_adj(a.oom_score_adj)
    node_setup.raise_nofile(a.max_open_files)
    if a.bootstrap_kubeconfig and a.kubeconfig:
        node_setup.bootstrap_client_cert(a.kubeconfig, a.bootstrap_kubeconfig,
                                         a.cert_dir or os.path.join(a.root_dir, "pki"), a.node_name)
    from ..client import Client
    from ..kubelet.kubelet import Kubelet, KubeletConfig
    labels = dict(kv.split("=", 1) for kv in a.node_labels.split(",") if "=" in kv)
    taints = []
    for t in filter(None, a.register_with_taints.split(",")):
        kv, eff = t.split(":")
        k, _, v = kv.partition("=")
        taints.append({"key": k, "value": v, "effect": eff})
    cfg = KubeletConfig(node_name=a.node_name, root_dir=a.root_dir,
                        plugins_dir=a.device_plugin_dir or os.path.join(a.root_dir, "device-plugin", "plugins"),
                        v1beta1_socket=a.device_plugin_v1beta1_socket, cri_socket=a.container_runtime_endpoint,
                        address=a.address, port=a.port, node_ip=a.node_ip, node_status_update_frequency=a.node_status_update_frequency,
                        relist_period=a.pleg_relist_period, max_pods=a.max_pods, node_labels=labels,
                        prioritize_device_pods=a.prioritize_device_pods == "true",
                        register_with_taints=taints, feature_gates=a.feature_gates, chaos_chance=a.chaos_chance,
                        pod_manifest_path=a.pod_manifest_path, file_check_frequency=a.file_check_frequency,
                        bootstrap_checkpoint_path=a.bootstrap_checkpoint_path,
                        gpu_stats_backend=a.gpu_stats_backend,
                        cluster_dns=[x for x in a.cluster_dns.split(",") if x], cluster_domain=a.cluster_domain,
                        resolv_conf=a.resolv_conf,
                        maximum_dead_containers_per_container=a.maximum_dead_containers_per_container,
                        maximum_dead_containers=a.maximum_dead_containers,
                        minimum_container_ttl_duration=a.minimum_container_ttl_duration,
                        eviction_hard=a.eviction_hard, eviction_soft=a.eviction_soft,
                        eviction_soft_grace_period=a.eviction_soft_grace_period,
                        eviction_minimum_reclaim=a.eviction_minimum_reclaim,
                        eviction_pressure_transition_period=a.eviction_pressure_transition_period,
                        eviction_max_pod_grace_period=a.eviction_max_pod_grace_period,
                        kube_reserved=a.kube_reserved, system_reserved=a.system_reserved,
                        enforce_node_allocatable=a.enforce_node_allocatable, cgroup_root=a.cgroup_root,
                        allowed_unsafe_sysctls=[x for x in a.experimental_allowed_unsafe_sysctls.split(",") if x],
                        cpu_manager_policy=a.cpu_manager_policy, cpu_manager_reconcile_period=a.cpu_manager_reconcile_period,
                        image_gc_high_threshold=a.image_gc_high_threshold, image_gc_low_threshold=a.image_gc_low_threshold,
                        minimum_image_ttl_duration=a.minimum_image_ttl_duration,
                        config_file=a.config, dynamic_config_dir=a.dynamic_config_dir,
                        cloud_provider=a.cloud_provider, cloud_config=a.cloud_config, volume_plugin_dir=a.volume_plugin_dir,
                        enable_controller_attach_detach=a.enable_controller_attach_detach == "true",
                        tls_cert_file=a.tls_cert_file, tls_private_key_file=a.tls_private_key_file,
                        client_ca_file=a.client_ca_file, anonymous_auth=a.anonymous_auth == "true",
                        authentication_token_webhook=a.authentication_token_webhook,
                        authorization_mode=a.authorization_mode, cert_dir=a.cert_dir,
                        rotate_certificates=a.rotate_certificates, rotate_server_certificates=a.rotate_server_certificates,
                        enable_server=a.enable_server, enable_debugging_handlers=a.enable_debugging_handlers,
                        read_only_port=a.read_only_port, healthz_port=a.healthz_port,
                        healthz_bind_address=a.healthz_bind_address, manifest_url=a.manifest_url,
                        manifest_url_header=dict(h.split(":", 1) for h in a.manifest_url_header.split(",") if ":" in h),
                        http_check_frequency=a.http_check_frequency, sync_frequency=a.sync_frequency,
                        register_node=a.register_node, register_schedulable=a.register_schedulable,
                        pod_cidr=a.pod_cidr, provider_id=a.provider_id, allow_privileged=a.allow_privileged,
                        host_network_sources=a.host_network_sources, host_pid_sources=a.host_pid_sources,
                        host_ipc_sources=a.host_ipc_sources, pods_per_core=a.pods_per_core,
                        serialize_image_pulls=a.serialize_image_pulls, registry_qps=a.registry_qps,
                        registry_burst=a.registry_burst, event_qps=a.event_qps, event_burst=a.event_burst,
                        runtime_request_timeout=a.runtime_request_timeout, image_service_endpoint=a.image_service_endpoint,
                        keep_terminated_pod_volumes=a.keep_terminated_pod_volumes,
                        volume_stats_agg_period=a.volume_stats_agg_period, cpu_cfs_quota=a.cpu_cfs_quota,
                        protect_kernel_defaults=a.protect_kernel_defaults, seccomp_profile_root=a.seccomp_profile_root,
                        cgroup_driver=a.cgroup_driver)

    async def mk():
        smi = None
        if a.gpu_stats_backend != "none":
            from ..smi import open_backend
            try:
                smi = open_backend(a.gpu_stats_backend)
            except Exception as e:
                logging.getLogger("amdkube.kubelet").warning("no GPU stats backend: %s", e)
        return await Kubelet(_client(a, qps=a.kube_api_qps, burst=a.kube_api_burst, chaos=a.chaos_chance), cfg,
                             smi_backend=smi).start()
    if a.runonce:
        # runonce.go: static pods only, no API server; exit status says whether all came up
        if not a.pod_manifest_path:
            raise SystemExit("--runonce needs --pod-manifest-path")
        from ..kubelet.runonce import NullClient, run_once, start_standalone

        async def once():
            k = await start_standalone(Kubelet(NullClient(), cfg))
            try:
                res = await run_once(k)
            finally:
                await k.volume_manager.stop()
            for r in res:
                print(json.dumps(r))
            return 0 if all(not r["error"] for r in res) else 1
        return asyncio.run(once())
    _run_forever(mk)


def rocshim(argv):
    ap = argparse.ArgumentParser("amdkube rocshim")
    ap.add_argument("--listen", default="/var/run/amdkube/rocshim.sock")
    ap.add_argument("--state-dir", default="/var/lib/amdkube/rocshim")
    ap.add_argument("--hooks-dir", default="/usr/share/containers/docker/hooks.d")
    ap.add_argument("--isolation", default="auto", choices=("env", "landlock", "userns", "namespaces", "auto"),
                    help="device isolation: auto probes the node (namespaces > userns > landlock > env)")
    ap.add_argument("--network-plugin", default="host", choices=("host", "cni", "kubenet"),
                    help="kubenet: pod network namespaces on the amdkube-bridge CNI plugin (cbr0 + host-local IPAM)")
    ap.add_argument("--pod-namespaces", action="store_true",
                    help="non-hostNetwork pods get their own net/ipc/uts namespaces (privileged; implied by kubenet)")
    ap.add_argument("--bridge", default="cbr0")
    ap.add_argument("--network-plugin-mtu", type=int, default=1460)
    ap.add_argument("--cni-conf-dir", default="/etc/cni/net.d")
    ap.add_argument("--cni-bin-dir", default=None, help="default: /opt/cni/bin plus amdkube's bundled plugins")
    ap.add_argument("--node-ip", default="127.0.0.1")
    ap.add_argument("--registry-dir", default=None,
                    help="directory standing in for image registries (<host>/<repo>/<tag>/, optional <host>/auth.json)")
    ap.add_argument("--insecure-registry", action="append", default=[],
                    help="registry host[:port] pulled over plain http (loopback registries always are), as dockerd's flag")
    ap.add_argument("--registry-ca", default=None, help="CA bundle for https registries")
    ap.add_argument("--cgroup-driver", default="cgroupfs", choices=("cgroupfs", "systemd"),
                    help="systemd: pods are slices and containers transient scopes, created over systemd's D-Bus API "
                         "(must match the kubelet's --cgroup-driver)")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "rocshim")
    from ..runtime import RocShim
    from ..runtime.images import NATIVE_BIN
    from ..runtime.network import CNINetwork, HostNetwork, KubenetNetwork
    if a.network_plugin == "kubenet":
        bins = a.cni_bin_dir.split(",") if a.cni_bin_dir else [os.path.join(NATIVE_BIN, "cni"), "/opt/cni/bin"]
        net = KubenetNetwork(bins, a.state_dir, a.bridge, a.network_plugin_mtu, a.node_ip)
    elif a.network_plugin == "cni":
        bins = a.cni_bin_dir.split(",") if a.cni_bin_dir else ["/opt/cni/bin", os.path.join(NATIVE_BIN, "cni")]
        net = CNINetwork(a.cni_conf_dir, bins, a.node_ip)
    else:
        net = HostNetwork(a.node_ip)

    async def mk():
        return await RocShim(a.listen, a.state_dir, a.hooks_dir, a.isolation, network=net,
                             pod_namespaces=a.pod_namespaces or a.network_plugin == "kubenet",
                             registry_dir=a.registry_dir, insecure_registries=a.insecure_registry,
                             registry_ca=a.registry_ca, cgroup_driver=a.cgroup_driver).start()
    _run_forever(mk)


def device_plugin(argv):
    ap = argparse.ArgumentParser("amdkube amd-device-plugin")
    ap.add_argument("--backend", default="auto", help="amdsmi|sysfs|fake|auto")
    ap.add_argument("--fixture", default=None)
    ap.add_argument("--plugins-dir", default="/var/lib/kubelet/device-plugin/plugins")
    ap.add_argument("--resource-name", default="amd.com/gpu")
    ap.add_argument("--health-interval", type=float, default=10.0)
    ap.add_argument("--health-probe", default="none", choices=("none", "hbm"))
    ap.add_argument("--max-gpus", type=int, default=None, help="advertise only the first N physical GPUs")
    ap.add_argument("--resource-naming", default="single", choices=("single", "mixed"),
                    help="partitioned GPUs: single=amd.com/gpu for all, mixed=amd.com/<cpx>_<nps> per partition type")
    ap.add_argument("--partition", default=None, help="fake backend only: compute/memory mode, e.g. CPX/NPS2")
    ap.add_argument("--register-v1beta1", default=None, help="kubelet.sock of an upstream v1beta1 kubelet")
    ap.add_argument("--health-state-file", default=None,
                    help="checkpoint of RAS baselines and GPU faults (default: <plugins-dir>/../amdkube-gpu-health.json; "
                         "'' keeps health state in memory only)")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "amd-device-plugin")
    state = a.health_state_file if a.health_state_file is not None else \
        os.path.join(os.path.dirname(os.path.abspath(a.plugins_dir)), "amdkube-gpu-health.json")
    from ..deviceplugin.amd import make_plugins
    from ..smi import open_backend

    class _Group:
        def __init__(self, plugins):
            self.plugins = plugins

        async def stop(self):
            for p in self.plugins:
                await p.stop()

    async def mk():
        backend = open_backend(a.backend, a.fixture, a.max_gpus, a.partition)
        plugins = make_plugins(backend, a.resource_naming, a.resource_name, plugins_dir=a.plugins_dir,
                               health_interval=a.health_interval, health_probe=a.health_probe,
                               health_state=state or None)
        for p in plugins:
            await p.start()
            if a.register_v1beta1:
                await p.register_v1beta1(a.register_v1beta1)
        return _Group(plugins)
    _run_forever(mk)


def gpu_health(argv):
    """`amdkube gpu-health show|reset [DEVICE_ID…|all]`: the device plugin's GPU fault
    checkpoint, and the operator's way to put a repaired GPU back into service."""
    ap = argparse.ArgumentParser("amdkube gpu-health")
    ap.add_argument("action", choices=("show", "reset"))
    ap.add_argument("devices", nargs="*", default=[])
    ap.add_argument("--state-file", default="/var/lib/kubelet/device-plugin/amdkube-gpu-health.json")
    a = ap.parse_args(argv)
    if a.action == "show":
        try:
            with open(a.state_file) as f:
                gpus = (json.load(f) or {}).get("gpus") or {}
        except FileNotFoundError:
            gpus = {}
        for did, ent in sorted(gpus.items()):
            print(f"{did}\t{'Unhealthy: ' + ent['sticky'] if ent.get('sticky') else 'Healthy'}")
        return 0
    if not a.devices:
        ap.error("reset needs device IDs or 'all'")
    from ..smi.health import request_reset
    request_reset(a.state_file, a.devices)
    print(f"reset requested for {', '.join(a.devices)} (applied on the plugin's next health check)")
    return 0


def addon_manager(argv):
    """cluster/addons/addon-manager/kube-addons.sh as a daemon (amdkube/addons.py). The reference's
    environment knobs are flags here, with the environment as the default."""
    ap = argparse.ArgumentParser("amdkube addon-manager")
    ap.add_argument("--server", default="http://127.0.0.1:8080")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--addon-path", default=os.environ.get("ADDON_PATH", "/etc/kubernetes/addons"))
    ap.add_argument("--admission-controls-path", default="/etc/kubernetes/admission-controls")
    ap.add_argument("--namespace-manifest", default=None, help="the kube-system Namespace manifest (/opt/namespace.yaml)")
    ap.add_argument("--check-interval", type=float,
                    default=float(os.environ.get("TEST_ADDON_CHECK_INTERVAL_SEC", "60")))
    ap.add_argument("--leader-election", default=os.environ.get("ADDON_MANAGER_LEADER_ELECTION", "true"),
                    choices=("true", "false"))
    ap.add_argument("--once", action="store_true", help="bootstrap, one ensure+reconcile pass, exit")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "addon-manager")
    from ..addons import AddonManager

    def mk_mgr():
        return AddonManager(_client(a), a.addon_path, a.admission_controls_path, a.check_interval,
                            leader_election=a.leader_election == "true", namespace_manifest=a.namespace_manifest)
    if a.once:
        async def once():
            mgr = mk_mgr()
            await mgr.bootstrap(30.0)
            await mgr.sync_once()
            await mgr.client.close()
        asyncio.run(once())
        return 0

    async def mk():
        return await mk_mgr().start()
    _run_forever(mk)


def node_problem_detector(argv):
    """node-problem-detector with the system-log monitors of deploy/node-problem-detector
    (monitoring/problemdetector.py); flags as in npd.yaml:46-51 and the reference's NPD e2e."""
    ap = argparse.ArgumentParser("amdkube node-problem-detector")
    ap.add_argument("--server", default="http://127.0.0.1:8080")
    ap.add_argument("--apiserver-override", default=None, help="URL of the apiserver (?inClusterConfig=false is ignored)")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--hostname-override", default=os.environ.get("NODE_NAME") or socket.gethostname())
    ap.add_argument("--system-log-monitors", default="", help="comma-separated monitor configs")
    ap.add_argument("--gpu-health-state", default="/var/lib/kubelet/device-plugin/amdkube-gpu-health.json",
                    help="the AMD device plugin's health checkpoint; gpuFault rules report into it ('' = off)")
    ap.add_argument("--resync-period", type=float, default=10.0)
    ap.add_argument("--logtostderr", action="store_true")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "node-problem-detector")
    if a.apiserver_override:
        a.server = a.apiserver_override.split("?", 1)[0]
    from ..monitoring.problemdetector import MonitorConfig, NodeProblemDetector
    configs = [MonitorConfig.load(p) for p in a.system_log_monitors.split(",") if p]
    if not configs:
        ap.error("no --system-log-monitors")

    async def mk():
        return await NodeProblemDetector(_client(a), a.hostname_override, configs, a.gpu_health_state or None,
                                         resync=a.resync_period).start()
    _run_forever(mk)


def cluster_proportional_autoscaler(argv):
    """cluster/addons/dns-horizontal-autoscaler (clusteraddons/proportional.py)."""
    ap = argparse.ArgumentParser("amdkube cluster-proportional-autoscaler")
    ap.add_argument("--server", default="http://127.0.0.1:8080")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--namespace", default=os.environ.get("MY_POD_NAMESPACE", "kube-system"))
    ap.add_argument("--configmap", required=True, help="ConfigMap holding the linear / ladder params")
    ap.add_argument("--target", required=True, help="Deployment/<name>, ReplicationController/<name> or ReplicaSet/<name>")
    ap.add_argument("--default-params", default="", help='JSON, e.g. {"linear":{"coresPerReplica":256,"nodesPerReplica":16}}')
    ap.add_argument("--poll-period-seconds", type=float, default=10.0)
    ap.add_argument("--logtostderr", default="true")
    ap.add_argument("-v", "--v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "cluster-proportional-autoscaler")
    from ..clusteraddons.proportional import ProportionalAutoscaler

    class _Runner:
        def __init__(self, pa):
            self.stop_ev = asyncio.Event()
            self.task = asyncio.create_task(pa.run(self.stop_ev))

        async def stop(self):
            self.stop_ev.set()
            await self.task

    async def mk():
        return _Runner(ProportionalAutoscaler(_client(a), a.namespace, a.configmap, a.target, a.default_params,
                                              a.poll_period_seconds))
    _run_forever(mk)


def ip_masq_agent(argv):
    """cluster/addons/ip-masq-agent (clusteraddons/ipmasq.py)."""
    ap = argparse.ArgumentParser("amdkube ip-masq-agent")
    ap.add_argument("--config", default="/etc/config/ip-masq-agent")
    ap.add_argument("--dry-run", action="store_true", help="render the chain without changing the host's tables")
    ap.add_argument("-v", "--v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "ip-masq-agent")
    from ..clusteraddons.ipmasq import MasqAgent

    class _Runner:
        def __init__(self, agent):
            self.stop_ev = asyncio.Event()
            self.task = asyncio.create_task(agent.run(self.stop_ev))

        async def stop(self):
            self.stop_ev.set()
            await self.task

    async def mk():
        return _Runner(MasqAgent(a.config, dry_run=True if a.dry_run else None))
    _run_forever(mk)


def dashboard(argv):
    """cluster/addons/dashboard (clusteraddons/dashboard.py)."""
    ap = argparse.ArgumentParser("amdkube dashboard")
    ap.add_argument("--server", "--apiserver-host", dest="server", default="http://127.0.0.1:8080")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--port", type=int, default=9090, help="HTTP port (kubernetes-dashboard's --insecure-port)")
    ap.add_argument("--address", default="0.0.0.0")
    ap.add_argument("--log-store-url", default="", help="the log store for the Logs view, e.g. http://elasticsearch-logging:9200")
    ap.add_argument("-v", "--v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "dashboard")
    from aiohttp import web
    from ..clusteraddons.dashboard import Dashboard

    class _Runner:
        async def start(self):
            self.runner = web.AppRunner(Dashboard(_client(a), a.log_store_url).app())
            await self.runner.setup()
            await web.TCPSite(self.runner, a.address, a.port).start()
            return self

        async def stop(self):
            await self.runner.cleanup()

    async def mk():
        return await _Runner().start()
    _run_forever(mk)


def log_store(argv):
    """The elasticsearch-logging service of cluster/addons/fluentd-elasticsearch (clusterlogging/store.py)."""
    ap = argparse.ArgumentParser("amdkube log-store")
    ap.add_argument("--data-dir", default="/data")
    ap.add_argument("--port", type=int, default=9200)
    ap.add_argument("--address", default="0.0.0.0")
    ap.add_argument("--retention-days", type=int, default=7)
    ap.add_argument("-v", "--v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "log-store")
    from aiohttp import web
    from ..clusterlogging.store import LogStore, app

    class _Runner:
        async def start(self):
            self.store = LogStore(a.data_dir, a.retention_days)
            self.runner = web.AppRunner(app(self.store))
            await self.runner.setup()
            await web.TCPSite(self.runner, a.address, a.port).start()
            self.task = asyncio.create_task(self._curate())
            return self

        async def _curate(self):
            while True:
                self.store.enforce_retention()
                await asyncio.sleep(3600)

        async def stop(self):
            self.task.cancel()
            await self.runner.cleanup()

    async def mk():
        return await _Runner().start()
    _run_forever(mk)


def log_shipper(argv):
    """The fluentd DaemonSet of cluster/addons/fluentd-elasticsearch (clusterlogging/shipper.py)."""
    ap = argparse.ArgumentParser("amdkube log-shipper")
    ap.add_argument("--server", default="http://127.0.0.1:8080")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--elasticsearch-url", default="http://elasticsearch-logging:9200")
    ap.add_argument("--containers-glob", default="/var/log/containers/*.log")
    ap.add_argument("--component-log", action="append", default=[], help="PATH[:TAG] of a glog-format log, repeatable")
    ap.add_argument("--pos-file", default="/var/log/amdkube-log-shipper.pos")
    ap.add_argument("--node-name", default=os.environ.get("NODE_NAME") or socket.gethostname())
    ap.add_argument("--flush-interval", type=float, default=5.0)
    ap.add_argument("-v", "--v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "log-shipper")
    from ..clusterlogging.shipper import Shipper

    class _Runner:
        def __init__(self, sh):
            self.stop_ev = asyncio.Event()
            self.task = asyncio.create_task(sh.run(self.stop_ev))

        async def stop(self):
            self.stop_ev.set()
            await self.task

    async def mk():
        return _Runner(Shipper(a.elasticsearch_url, a.containers_glob, a.component_log, a.pos_file, _client(a), a.node_name,
                               flush_interval=a.flush_interval))
    _run_forever(mk)


def exporter(argv):
    ap = argparse.ArgumentParser("amdkube amdgpu-exporter")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--port", type=int, default=9400)
    ap.add_argument("--address", default="0.0.0.0")
    ap.add_argument("--node-name", default=socket.gethostname())
    ap.add_argument("--kubelet-url", default=None)
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "amdgpu-exporter")
    from ..monitoring.exporter import Exporter
    from ..smi import open_backend

    async def mk():
        return await Exporter(open_backend(a.backend), a.node_name, a.kubelet_url).start(a.address, a.port)
    _run_forever(mk)


def metrics_server(argv):
    """Resource metrics API (metrics.k8s.io) and the custom metrics API (custom.metrics.k8s.io:
    gpu_utilization / gpu_memory_used_bytes / gpu_count per pod and node) behind the aggregator:
    register an APIService per group pointing at a Service whose endpoints reach --secure-port."""
    ap = argparse.ArgumentParser("amdkube metrics-server")
    ap.add_argument("--master", "--server", dest="server", default="http://127.0.0.1:8080")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--token", default=None)
    ap.add_argument("--bind-address", default="0.0.0.0")
    ap.add_argument("--secure-port", type=int, default=443)
    ap.add_argument("--tls-cert-file", default=None)
    ap.add_argument("--tls-private-key-file", default=None)
    ap.add_argument("--requestheader-client-ca-file", default=None)
    ap.add_argument("--requestheader-allowed-names", default="")
    ap.add_argument("--metric-resolution", type=float, default=60.0, help="seconds between kubelet scrapes")
    ap.add_argument("--kubelet-https", default="false", choices=("true", "false"))
    ap.add_argument("--kubelet-insecure-tls", action="store_true")
    ap.add_argument("--authorization-always-allow", action="store_true", help="skip authn/authz (testing only)")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "metrics-server")
    from ..metrics import MetricsServer

    async def mk():
        kssl = None
        if a.kubelet_https == "true" and a.kubelet_insecure_tls:
            import ssl
            kssl = ssl.create_default_context()
            kssl.check_hostname, kssl.verify_mode = False, ssl.CERT_NONE
        return await MetricsServer(_client(a), a.metric_resolution, a.requestheader_client_ca_file,
                                   [x for x in a.requestheader_allowed_names.split(",") if x], a.tls_cert_file,
                                   a.tls_private_key_file, "https" if a.kubelet_https == "true" else "http", kssl,
                                   authorize=not a.authorization_always_allow).start(a.bind_address, a.secure_port)
    _run_forever(mk)


def hollow_node(argv):
    ap = argparse.ArgumentParser("amdkube hollow-node")
    ap.add_argument("--server", default="http://127.0.0.1:8080")
    ap.add_argument("--name-prefix", default="hollow-node")
    ap.add_argument("--count", type=int, default=1)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--run-seconds", type=float, default=None)
    ap.add_argument("--partition", default="SPX/NPS1", help="simulated compute/memory partition mode, e.g. CPX/NPS2")
    ap.add_argument("--resource-naming", default="single", choices=("single", "mixed"))
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "hollow-node")
    from ..hollow.hollow_node import HollowNode

    class Group:
        def __init__(self, nodes):
            self.nodes = nodes

        async def stop(self):
            for n in self.nodes:
                await n.stop()

    async def mk():
        nodes = [await HollowNode(a.server, f"{a.name_prefix}-{i}", a.gpus, a.run_seconds, partition=a.partition,
                                  resource_naming=a.resource_naming).start() for i in range(a.count)]
        return Group(nodes)
    _run_forever(mk)


def proxy(argv):
    ap = argparse.ArgumentParser("amdkube proxy")
    ap.add_argument("--master", "--server", dest="server", default="http://127.0.0.1:8080")
    ap.add_argument("--kubeconfig", default=None, help="kubeconfig with the server, CA and credentials")
    ap.add_argument("--token", default=None, help="bearer token for the apiserver")
    ap.add_argument("--proxy-mode", default="userspace", choices=("userspace", "iptables", "ipvs"))
    ap.add_argument("--ipvs-scheduler", default="rr")
    ap.add_argument("--bind-address", default="0.0.0.0", help="node address NodePorts listen on")
    ap.add_argument("--cluster-cidr", default="")
    ap.add_argument("--iptables-sync-period", type=float, default=30.0)
    ap.add_argument("--iptables-min-sync-period", type=float, default=0.0)
    ap.add_argument("--healthz-port", type=int, default=10256)
    ap.add_argument("--iptables-dump-file", default=None, help="write every rendered ruleset here (dry-run inspection)")
    tf = lambda v: str(v).lower() in ("true", "1", "yes")   # noqa: E731
    ap.add_argument("--config", default=None, help="KubeProxyConfiguration file (its fields override the flags)")
    ap.add_argument("--write-config-to", default=None, help="write the effective configuration here and exit")
    ap.add_argument("--cleanup", "--cleanup-iptables", "--cleanup-ipvs", dest="cleanup", action="store_true",
                    help="remove the rules this proxy installs and exit")
    ap.add_argument("--masquerade-all", type=tf, default=False)
    ap.add_argument("--iptables-masquerade-bit", type=int, default=14)
    ap.add_argument("--ipvs-sync-period", type=float, default=30.0)
    ap.add_argument("--ipvs-min-sync-period", type=float, default=0.0)
    ap.add_argument("--healthz-bind-address", default="127.0.0.1")
    ap.add_argument("--metrics-bind-address", default="127.0.0.1:10249")
    ap.add_argument("--hostname-override", default="")
    ap.add_argument("--oom-score-adj", type=int, default=-999)
    ap.add_argument("--udp-timeout", type=float, default=0.25, help="userspace UDP idle timeout (s)")
    ap.add_argument("--conntrack-max-per-core", type=int, default=32768)
    ap.add_argument("--conntrack-min", type=int, default=131072)
    ap.add_argument("--conntrack-max", type=int, default=0)
    ap.add_argument("--conntrack-tcp-timeout-established", type=float, default=86400.0, help="seconds")
    ap.add_argument("--conntrack-tcp-timeout-close-wait", type=float, default=3600.0, help="seconds")
    ap.add_argument("--kube-api-qps", type=float, default=5.0)
    ap.add_argument("--kube-api-burst", type=int, default=10)
    for flag in ("--kube-api-content-type", "--config-sync-period", "--proxy-port-range", "--resource-container",
                 "--profiling", "--feature-gates"):
        ap.add_argument(flag, default=None, help=argparse.SUPPRESS)
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "proxy")
    from ..proxy import config_file
    if a.config:
        config_file.apply(a, config_file.load(a.config))
    if a.write_config_to:
        config_file.write(a, a.write_config_to)
        print(f"Wrote configuration to: {a.write_config_to}")
        return 0
    if a.cleanup:       # server.go CleanupAndExit
        from ..proxy import iptables as ipt
        rules = ipt.cleanup(dry_run=os.geteuid() != 0)
        if shutil.which("ipvsadm") and os.geteuid() == 0:
            subprocess.run(["ipvsadm", "-C"], capture_output=True)
            subprocess.run(["ip", "link", "del", "kube-ipvs0"], capture_output=True)
        print(rules, end="")
        return 0
    from ..kubelet.node_setup import apply_oom_score_adj
    apply_oom_score_adj(a.oom_score_adj)
    config_file.apply_conntrack(a)
    from ..proxy import ProxyServer
    mhost, _, mport = a.metrics_bind_address.rpartition(":")
    sync, min_sync = (a.ipvs_sync_period, a.ipvs_min_sync_period) if a.proxy_mode == "ipvs" else \
        (a.iptables_sync_period, a.iptables_min_sync_period)

    async def mk():
        return await ProxyServer(_client(a, qps=a.kube_api_qps, burst=a.kube_api_burst), a.proxy_mode, a.bind_address,
                                 a.cluster_cidr, sync, min_sync, a.healthz_port, a.iptables_dump_file,
                                 ipvs_scheduler=a.ipvs_scheduler, masquerade_all=a.masquerade_all,
                                 masquerade_bit=a.iptables_masquerade_bit, healthz_address=a.healthz_bind_address,
                                 udp_idle_timeout=a.udp_timeout, metrics_address=(mhost or "127.0.0.1", int(mport or 0)),
                                 hostname=a.hostname_override or socket.gethostname()).start()
    _run_forever(mk)


def dns(argv):
    """Cluster DNS addon (kube-dns equivalent, amdkube/dns)."""
    ap = argparse.ArgumentParser("amdkube dns")
    ap.add_argument("--master", "--server", dest="server", default="http://127.0.0.1:8080")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--token", default=None)
    ap.add_argument("--domain", "--cluster-domain", dest="domain", default="cluster.local")
    ap.add_argument("--dns-bind-address", default="127.0.0.1")
    ap.add_argument("--dns-port", type=int, default=53)
    ap.add_argument("--upstream", default=None, help="comma-separated upstream servers (default: the host's resolv.conf)")
    ap.add_argument("-conf", "--conf", dest="conf", default=None,
                    help="a CoreDNS Corefile (dns/corefile.py): its kubernetes zone, proxy upstreams and port; "
                         "--domain/--upstream/--dns-port given explicitly win")
    ap.add_argument("-v", type=int, default=0)
    a = ap.parse_args(argv)
    klog.setup(a.v, "dns")
    from ..dns import DNSServer
    up = [x for x in a.upstream.split(",") if x] if a.upstream is not None else None
    if a.conf:
        from ..dns.corefile import parse
        with open(a.conf) as f:
            cf = parse(f.read())
        given = set(argv)
        if not given & {"--domain", "--cluster-domain"}:
            a.domain = cf["domain"]
        if "--dns-port" not in given:
            a.dns_port = cf["port"]
        if up is None:
            up = cf["upstream"]

    async def mk():
        return await DNSServer(_client(a), a.domain, a.dns_bind_address, a.dns_port, up).start()
    _run_forever(mk)


def local_up(argv):
    """hack/local-up-cluster.sh equivalent: every component as its own process."""
    ap = argparse.ArgumentParser("amdkube local-up")
    ap.add_argument("--base-dir", default="/tmp/amdkube-local")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--max-gpus", type=int, default=None)
    ap.add_argument("--isolation", default="auto")
    ap.add_argument("--no-gpus", action="store_true")
    ap.add_argument("--exporter-port", type=int, default=9400)
    a = ap.parse_args(argv)
    b = a.base_dir
    os.makedirs(os.path.join(b, "logs"), exist_ok=True)
    server = f"http://127.0.0.1:{a.port}"
    py = [sys.executable, "-m", "amdkube"]
    procs = []

    def spawn(name, args):
        logf = open(os.path.join(b, "logs", f"{name}.log"), "ab")
        p = subprocess.Popen(py + args, stdout=logf, stderr=subprocess.STDOUT)
        procs.append((name, p))
        return p

    def wait_http(url, timeout=30):
        import urllib.request
        end = time.time() + timeout
        while time.time() < end:
            try:
                urllib.request.urlopen(url, timeout=1)
                return True
            except Exception:
                time.sleep(0.1)
        return False

    spawn("apiserver", ["apiserver", "--port", str(a.port), "--data-dir", os.path.join(b, "store")])
    if not wait_http(server + "/healthz"):
        raise SystemExit("apiserver did not come up; see " + os.path.join(b, "logs", "apiserver.log"))
    spawn("controller-manager", ["controller-manager", "--server", server])
    spawn("scheduler", ["scheduler", "--server", server, "--port", "0"])
    spawn("proxy", ["proxy", "--server", server, "--healthz-port", "0"])
    # cluster DNS: on :53 it is the pods' nameserver (root); otherwise it still serves on :10053
    dns_port = 53 if os.geteuid() == 0 else 10053
    spawn("dns", ["dns", "--server", server, "--dns-port", str(dns_port), "--dns-bind-address", "127.0.0.1"])
    dns_flags = ["--cluster-dns", "127.0.0.1", "--cluster-domain", "cluster.local"] if dns_port == 53 else []
    sock = os.path.join(b, "rocshim.sock")
    spawn("rocshim", ["rocshim", "--listen", sock, "--state-dir", os.path.join(b, "rocshim"), "--hooks-dir",
                      os.path.join(b, "hooks.d"), "--isolation", a.isolation])
    plugins = os.path.join(b, "device-plugin", "plugins")
    if not a.no_gpus:
        dp = ["amd-device-plugin", "--backend", a.backend, "--plugins-dir", plugins]
        if a.max_gpus:
            dp += ["--max-gpus", str(a.max_gpus)]
        spawn("amd-device-plugin", dp)
        spawn("amdgpu-exporter", ["amdgpu-exporter", "--backend", a.backend, "--port", str(a.exporter_port),
                                  "--kubelet-url", "http://127.0.0.1:10250"])
    for _ in range(100):
        if os.path.exists(sock):
            break
        time.sleep(0.1)
    spawn("kubelet", ["kubelet", "--server", server, "--root-dir", os.path.join(b, "kubelet"), "--device-plugin-dir", plugins,
                      "--container-runtime-endpoint", sock, "--gpu-stats-backend", "none" if a.no_gpus else a.backend,
                      "--read-only-port", "0", "--healthz-port", "0", "--fail-swap-on", "false"]
          + dns_flags)
    os.makedirs(os.path.expanduser("~/.amdkube"), exist_ok=True)
    json.dump({"server": server}, open(os.path.expanduser("~/.amdkube/config"), "w"))
    print(f"amdkube local cluster is running: {server}  (logs: {b}/logs)\n"
          f"  python -m amdkube kubectl get nodes\n  python -m amdkube kubectl run vadd --image rocm/vector-add --gpus 1 --restart Never",
          flush=True)
    stop = {"flag": False}
    signal.signal(signal.SIGTERM, lambda *_: stop.update(flag=True))
    try:
        while not stop["flag"]:
            for name, p in procs:
                if p.poll() is not None:
                    print(f"{name} exited with {p.returncode}; see {b}/logs/{name}.log", flush=True)
                    stop["flag"] = True
            time.sleep(0.5)
    except KeyboardInterrupt:
        pass
    finally:
        for name, p in reversed(procs):
            p.send_signal(signal.SIGTERM)
        for name, p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()


def kubeadm(argv):
    from ..kubeadm import main
    return main(argv)


COMPONENTS = {"etcd": etcd, "dns": dns, "kube-dns": dns, "kubeadm": kubeadm, "proxy": proxy, "kube-proxy": proxy, "apiserver": apiserver, "kube-apiserver": apiserver, "scheduler": scheduler, "kube-scheduler": scheduler,
              "controller-manager": controller_manager, "kube-controller-manager": controller_manager, "kubelet": kubelet,
              "rocshim": rocshim, "amd-device-plugin": device_plugin, "device-plugin": device_plugin,
              "gpu-health": gpu_health, "addon-manager": addon_manager, "node-problem-detector": node_problem_detector,
              "cluster-proportional-autoscaler": cluster_proportional_autoscaler, "ip-masq-agent": ip_masq_agent,
              "dashboard": dashboard, "log-store": log_store, "log-shipper": log_shipper,
              "amdgpu-exporter": exporter, "exporter": exporter, "hollow-node": hollow_node, "local-up": local_up,
              "metrics-server": metrics_server, "cloud-controller-manager": cloud_controller_manager,
              "gke-certificates-controller": gke_certificates_controller, "rktshim": rktshim}
from .gendocs import GENERATORS as _GENERATORS  # noqa: E402  (gendocs/genkubedocs/genman/genyaml)
COMPONENTS.update(_GENERATORS)

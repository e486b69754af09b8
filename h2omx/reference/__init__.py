"""CPU reference implementations (test oracle and CPU-only runs); see h2omx.backend."""

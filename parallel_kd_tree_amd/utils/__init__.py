"""Runtime services: generator, on-disk layout, CLI protocol, timing."""

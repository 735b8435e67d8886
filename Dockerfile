# ROCm 7 + PyTorch image with the gfx950 kernels built in-tree.
FROM rocm/pytorch:latest
WORKDIR /opt/foremast
COPY . .
RUN pip install --no-cache-dir fastapi uvicorn httpx prometheus_client pyyaml scipy \
 && PYTORCH_ROCM_ARCH=gfx950 python -c "import __graft_entry__ as g; g.build()"
ENV PYTHONPATH=/opt/foremast HSA_ENABLE_IPC_MODE_LEGACY=0
EXPOSE 8099 8000
CMD ["python", "-m", "foremast_amd.service"]

for r in 1 2; do
HSA_ALLOCATE_QUEUE_DEV_MEM=1 timeout -k 10 120 python3 -u tools/sync_ab.py --tag "ring VRAM" || exit 1
timeout -k 10 120 python3 -u tools/sync_ab.py --tag "ring host" || exit 1
done

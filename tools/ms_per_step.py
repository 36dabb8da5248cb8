"""Print ms_per_step of the bench JSON line read from stdin."""
import json
import sys

print(json.loads(sys.stdin.read())['ms_per_step'])

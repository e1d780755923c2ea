#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 9
bash tools/profile_session.sh "$@"
